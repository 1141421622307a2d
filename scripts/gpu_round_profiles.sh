cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/*
scripts/gpu_steps.sh \
 gputests 400 "python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 bench_c2 240 "python -u bench.py > gpurun_out/r1_bench_c2.json" \
 stats_c2 240 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/stats_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu-baseline --no-work" \
 pmc_c2 600 "scripts/pmc_passes.sh gpurun_out/pmc_c2 --config c2" \
 shards 240 "python -u scripts/shard_probe.py --shards 1 2 4 8 > gpurun_out/shard_probe_c2.jsonl" \
 bench_c4 300 "python -u bench.py --config c4 --steps 1 --warmup 0 > gpurun_out/r1_bench_c4.json" \
 stats_c4 240 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/stats_c4 -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-work"
