"""Per-kernel register / scratch / occupancy table of the render kernels (hipcc -Rpass-analysis).

    python scripts/resources.py [filter] [--tu spheres|spheres_global|cornell|full|full_dark|render ...] [-- extra hipcc flags]

The translation units (rt_k_*.hip, rt_render.hip) compile in parallel; --tu limits the run to some.
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
    tus = ["spheres", "spheres_global", "cornell", "full", "full_dark", "render"]
    if "--tu" in args:
        i = args.index("--tu")
        sel = [a for a in args[i + 1:] if a in tus]
        args = args[:i] + [a for a in args[i + 1:] if a not in tus]
        tus = sel
    filt = args[0] if args else ""
    csrc = f"{ROOT}/ray-tracing_amd/csrc"
    procs = []
    for tu in tus:
        src = f"{csrc}/rt_render.hip" if tu == "render" else f"{csrc}/rt_k_{tu}.hip"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-fno-fast-math", f"-I{ROOT}/include", "-c", src, "-o", "/dev/null",
               "-Rpass-analysis=kernel-resource-usage"] + extra
        procs.append(subprocess.Popen(cmd, stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, text=True))
    out = "\n".join(p.communicate()[1] for p in procs)
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
