"""Same-box A/B tool: every arm × every workload, interleaved passes, one JSON line per run.

    python bench/ab.py --arm "base:PENROZ_EXT_DIR=build_ab" --arm "new:" \
        --work headline --work gemma3-1b:8 --work decode:gpt2:64 --work "attn:--B 64 --T 1024 --H 12 --D 64" \
        --passes 2 --log gpurun_out/ab.jsonl

An arm is ``name:ENV=VAL ENV2=VAL2`` (empty env = the working tree as is). A baseline build is an
arm whose env sets ``PENROZ_EXT_DIR`` to a second in-tree build directory; a GEMM-table variant sets
``PENROZ_TUNED_GEMM_FILE``; ``AB_CWD=dir`` runs the arm from another in-tree checkout (e.g. the
previous commit's Python, ``git archive HEAD | tar -x -C ab_head`` with ``build_ext`` linked in). Workloads:

* ``headline`` — ``bench.py`` (GPT-2 124M, B = 64, T = 1024), 20 timed / 5 warmup steps;
* ``bench:<model>[:<batch>]`` / ``gemma3-1b[:<batch>]`` — ``bench.py --model …``;
* ``decode:<model>:<batch>`` — ``bench/bench_decode.py`` with the graph decode program;
* ``attn:<attn_bench.py args>`` — the flash-attention microbench.

Runs go arm-major inside a pass and passes repeat, so a drifting box clock shows up as a pass
difference rather than an arm difference. Every run has its own time limit; a failing run ends the
tool (exit 1) — nothing is retried. This replaces the per-round one-off ``gpu_*.sh`` A/B scripts.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_arm(spec: str) -> tuple[str, dict]:
    name, _, env = spec.partition(":")
    kv = {}
    for tok in shlex.split(env):
        k, _, v = tok.partition("=")
        if not k or not _:
            raise SystemExit(f"bad arm env {tok!r} in {spec!r} (want ENV=VAL)")
        kv[k] = v
    return name or "arm", kv


def work_cmd(work: str, steps: int, warmup: int) -> tuple[list[str], int]:
    """(argv, time limit s) of one workload."""
    py = sys.executable
    if work == "headline":
        return [py, "bench.py", "--steps", str(steps), "--warmup", str(warmup), "--ref-steps", "0"], 240
    kind, _, rest = work.partition(":")
    if kind in ("bench", "gemma3-1b"):
        parts = rest.split(":") if rest else []
        model = "gemma3-1b" if kind == "gemma3-1b" else parts.pop(0)
        argv = [py, "bench.py", "--model", model, "--steps", str(max(3, steps // 4)), "--warmup", "2", "--ref-steps", "0"]
        if parts:
            argv += ["--batch", parts[0]]
        return argv, 400
    if kind == "decode":
        model, _, batch = rest.partition(":")
        return [py, "bench/bench_decode.py", "--model", model or "gpt2", "--batch", batch or "64"], 240
    if kind == "attn":
        return [py, "bench/attn_bench.py"] + shlex.split(rest) + ["--iters", "10"], 120
    raise SystemExit(f"unknown workload {work!r}")


def headline_number(stdout: str) -> dict:
    """The last JSON line of a run, reduced to the fields an A/B compares."""
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    if not lines:
        return {}
    d = json.loads(lines[-1])
    keep = ("ms_per_step", "value", "mfu_bf16_dense", "fwd_us", "fwd_v3_us", "bwd_us", "fwd_TF", "fwd_v3_TF", "bwd_TF")
    return {k: d[k] for k in keep if k in d}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--arm", action="append", required=True, help="name:ENV=VAL ... (repeatable)")
    ap.add_argument("--work", action="append", default=None, help="workload (repeatable; default headline)")
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--log", default=os.path.join(ROOT, "gpurun_out", "ab.jsonl"))
    args = ap.parse_args(argv)
    arms = [parse_arm(a) for a in args.arm]
    works = args.work or ["headline"]
    os.makedirs(os.path.dirname(args.log), exist_ok=True)
    with open(args.log, "a") as logf:
        for p in range(1, args.passes + 1):
            for work in works:
                cmd, limit = work_cmd(work, args.steps, args.warmup)
                for name, env in arms:
                    env = dict(env)
                    cwd = os.path.join(ROOT, env.pop("AB_CWD")) if "AB_CWD" in env else ROOT
                    full = dict(os.environ, **env)
                    t0 = time.time()
                    r = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, cwd=cwd, env=full,
                                       capture_output=True, text=True)
                    rec = {"pass": p, "work": work, "arm": name, "env": env, "rc": r.returncode,
                           "wall_s": round(time.time() - t0, 1), **headline_number(r.stdout)}
                    logf.write(json.dumps(rec) + "\n")
                    logf.flush()
                    print(json.dumps(rec), flush=True)
                    if r.returncode != 0:
                        sys.stderr.write(r.stdout[-2000:] + r.stderr[-4000:])
                        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
