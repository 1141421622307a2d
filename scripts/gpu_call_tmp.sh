# round 6: C5 evidence on the final build (rocprofv3 kernel stats, bench line)
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
scripts/gpu_steps.sh \
  stats_c5 400 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stats_c5b -o c5 -- python3 $PWD/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-work" \
  bench_c5 600 "python -u bench.py --config c5 --steps 1 --warmup 1 > gpurun_out/r6_bench_c5_final.json"
