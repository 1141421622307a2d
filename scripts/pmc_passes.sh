#!/bin/bash
# PMC passes for a config's render kernel (the last pass: instruction-cache requests / misses) (one rocprofv3 run per counter group, --kernel-trace only;
# MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE need separate passes).
# usage: scripts/pmc_passes.sh <outdir> [bench args...]
out=$1; shift
args="$*"
set -e
mkdir -p "$out"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES" \
           "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/pass$i" -o p -- \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-work $args > "$out/pass$i.log" 2>&1
done
