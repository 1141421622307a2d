# round-6 evidence for the final C2 / C1 kernels and the GPU suite
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
scripts/gpu_steps.sh \
  gputest_final 900 "python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA -s" \
  smoke_final 300 "python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
rc=$?; [ $rc -ge 124 ] && exit $rc
scripts/gpu_round_profiles.sh r6 c2 c1
