#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "walks_output or closest_hits" --timeout 100 --timeout-method thread > gpurun_out/t.log 2>&1 || exit $?
for rep in 1 2; do
for b in 64 48 32 16 8; do
  echo "c4 box_first $b: $(RTAMD_BOX_FIRST=$b timeout -k 10 90 python -u bench.py --config c4 --spp 100 --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' ')" >> gpurun_out/bf.log
  echo "c3 box_first $b: $(RTAMD_BOX_FIRST=$b timeout -k 10 90 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' ')" >> gpurun_out/bf.log
done; done
