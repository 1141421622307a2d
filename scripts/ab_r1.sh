cd $GRAFT_REPO_ROOT
for i in 1 2; do
  echo "r1 c4: $(cd _ab_r1 && timeout -k 10 200 python bench.py --config c4 --spp 100 --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  echo "r2 c4 skel0: $(RTAMD_SKELETON=0 timeout -k 10 200 python bench.py --config c4 --spp 100 --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  echo "r2 c4 skel1: $(timeout -k 10 200 python bench.py --config c4 --spp 100 --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  echo "r1 c2: $(cd _ab_r1 && timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  echo "r2 c2: $(timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
