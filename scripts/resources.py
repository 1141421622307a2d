"""Per-kernel register / scratch / occupancy table of rt_render.hip (hipcc -Rpass-analysis).

    python scripts/resources.py [filter] [-- extra hipcc flags]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    filt = args[0] if args else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           "-fno-fast-math", f"-I{ROOT}/include", "-c", f"{ROOT}/ray-tracing_amd/csrc/rt_render.hip", "-o",
           "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: +([A-Za-z][\w \[\]/]*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        if filt and filt not in r["name"]:
            continue
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '?'):>3} agpr  scratch {r.get('ScratchSize [bytes/lane]', '?'):>4}"
              f"  occ {r.get('Occupancy [waves/SIMD]', '?')}  vspill {r.get('VGPRs Spill', '?'):>4}"
              f"  sspill {r.get('SGPRs Spill', '?'):>4}  lds {r.get('LDS Size [bytes/block]', '?'):>6}  {r['name'][:110]}")


if __name__ == "__main__":
    main()
