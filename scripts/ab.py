"""Same-box A/B harness (replaces the round-1..3 one-off shell scripts): build variants of the library
here, then time them against the working tree in ONE GPU call, alternating legs so that box-to-box
variance (up to 9 %) cancels.

Build (CPU, this container) — a self-contained copy of bench.py, scripts/, the package and its library:
    python scripts/ab.py build NAME [--rev REV] [--patch EDIT.py] [--flags "EXTRA HIPCC FLAGS"]
        --rev REV      a committed revision (git worktree under /tmp); default: the working tree
        --patch P.py   a python script run with the copied source dir as argv[1] (experiments not in
                       the tree yet)
        --flags F      extra hipcc flags (code-generation variants)
    -> _var_NAME/   (listed in .gitignore; it travels to the GPU box with the snapshot)

Time (GPU box) — one line per leg and repetition, also appended to gpurun_out/ab.log:
    python scripts/ab.py time [--bench "ARGS"] [--shards N ...] [--work] [--reps R] LEG [LEG ...]
        LEG = DIR[:VAR=VAL[,VAR=VAL...]]   DIR = . (the tree) or _var_NAME; VARs are RTAMD_* knobs
        --bench ARGS   bench.py arguments (default "--config c2"); reports the render kernel's ms per step
        --shards N..   run scripts/shard_probe.py instead (per-shard ms at those shard counts)
        --work         also the counting pass: work per sample, lane utilisation, tie redos
    e.g.  python scripts/ab.py time --bench "--config c4 --spp 100" . _var_x .:RTAMD_BOX_FIRST=8
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(a):
    src = f"/tmp/ab_src_{a.name}"
    shutil.rmtree(src, ignore_errors=True)
    if a.rev:
        wt = "/tmp/ab_worktree"
        # (the revision is resolved in the main repository: "HEAD" inside the worktree is the worktree's)
        sha = subprocess.run(["git", "-C", ROOT, "rev-parse", a.rev], check=True, capture_output=True,
                             text=True).stdout.strip()
        if not os.path.isdir(wt):
            subprocess.run(["git", "-C", ROOT, "worktree", "add", "-f", "--detach", wt, sha], check=True)
        subprocess.run(["git", "-C", wt, "checkout", "-q", "--detach", sha], check=True)
        base = wt
    else:
        base, sha = ROOT, ""
    os.makedirs(src)
    for d in ("ray-tracing_amd", "include"):
        shutil.copytree(os.path.join(base, d), os.path.join(src, d), ignore=shutil.ignore_patterns("build", "__pycache__"))
    if a.patch:
        subprocess.run([sys.executable, a.patch, src], check=True)
    log = os.path.join(src, "build.log")
    with open(log, "w") as f:  # (a stale library must never stand in for a failed build: the copy starts empty)
        r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(src, "ray-tracing_amd", "csrc"), f"EXTRA={a.flags}"],
                           stdout=f, stderr=subprocess.STDOUT)
    if r.returncode:
        print(open(log).read()[-3000:])
        sys.exit(f"build of _var_{a.name} failed")
    out = os.path.join(ROOT, f"_var_{a.name}")
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(os.path.join(out, "tests", "golden"))
    os.makedirs(os.path.join(out, "ray-tracing_amd", "build"))
    shutil.copy(os.path.join(base, "bench.py"), out)
    shutil.copytree(os.path.join(base, "scripts"), os.path.join(out, "scripts"))
    shutil.copytree(os.path.join(src, "ray-tracing_amd", "rtamd"), os.path.join(out, "ray-tracing_amd", "rtamd"))
    shutil.copy(os.path.join(src, "ray-tracing_amd", "build", "librtamd.so"), os.path.join(out, "ray-tracing_amd", "build"))
    shutil.copy(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.npz"), os.path.join(out, "tests", "golden"))
    what = (f"rev {a.rev} ({sha[:10]})" if a.rev else "working tree") + (f", patch {a.patch}" if a.patch else "") + (
        f", flags {a.flags}" if a.flags else "")
    print(f"_var_{a.name}: {what}")


def leg_env(leg):
    d, _, spec = leg.partition(":")
    env = dict(os.environ)
    for kv in filter(None, spec.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    return (ROOT if d in (".", "") else os.path.join(ROOT, d)), env


def run_leg(leg, a):
    d, env = leg_env(leg)
    if a.shards:
        cmd = [sys.executable, "-u", "scripts/shard_probe.py", "--shards", *map(str, a.shards), "--reps", "2"] + (
            a.bench.split() if a.bench else [])
    else:
        cmd = [sys.executable, "-u", "bench.py", "--steps", str(a.steps), "--warmup", "1", "--no-cpu-baseline"] + (
            [] if a.work else ["--no-work"]) + a.bench.split()
    t0 = time.time()
    r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=a.timeout)
    if r.returncode:
        return f"FAIL rc={r.returncode}: {r.stderr[-400:]}", r.returncode
    if a.shards:
        return " | ".join(re.findall(r"N=\d+: per-shard [0-9.]+ ms", r.stdout)), 0
    ks = re.findall(r"kernel ([0-9.]+) ms", r.stderr)
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    out = f"kernel {' '.join(ks)} ms, {line['ms_per_step']:.1f} ms/step ({time.time() - t0:.0f} s)"
    if a.work and line.get("work_per_sample"):
        w = line["work_per_sample"]
        out += (f"; per sample: wide {w.get('wide_nodes')} box {w.get('box_tests')} leaf {w.get('prim_tests')} "
                f"other {w.get('other_tests')} ties {w.get('tie_redos')}; util {line.get('lane_utilisation')}")
    return out, 0


def time_legs(a):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ab.log"), "a") as logf:
        logf.write(f"== ab.py time {a.bench or ''} shards={a.shards} legs={a.legs}\n")
        for rep in range(a.reps):
            for leg in a.legs:
                msg, rc = run_leg(leg, a)
                line = f"[{rep + 1}] {leg}: {msg}"
                print(line, flush=True)
                logf.write(line + "\n")
                logf.flush()
                if rc >= 124 or rc < 0 or rc in (134, 139):  # a fault or a limit: nothing more on the GPU
                    sys.exit(rc if rc > 0 else 1)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("build")
    b.add_argument("name")
    b.add_argument("--rev", default="")
    b.add_argument("--patch", default="")
    b.add_argument("--flags", default="")
    t = sub.add_parser("time")
    t.add_argument("legs", nargs="+")
    t.add_argument("--bench", default="--config c2")
    t.add_argument("--shards", type=int, nargs="*")
    t.add_argument("--work", action="store_true")
    t.add_argument("--reps", type=int, default=2)
    t.add_argument("--steps", type=int, default=2)
    t.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args()
    build(a) if a.cmd == "build" else time_legs(a)


if __name__ == "__main__":
    main()
