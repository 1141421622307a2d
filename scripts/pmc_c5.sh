#!/bin/bash
out=gpurun_out/pmc_c5
mkdir -p $out
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAVES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/pass$i" -o p -- \
    python bench.py --config c5 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --no-work > "$out/pass$i.log" 2>&1 || exit $?
done
