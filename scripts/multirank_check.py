"""Rehearsal of bench.py's multi-GPU paths on ONE GPU: torchrun with 2 and 3
ranks (every rank on cuda:0, gloo instead of RCCL, which refuses two ranks on
one device), and the launcher-free single-process path (rt_multi over 3 and
8 "devices" that are all cuda:0, peer copies), each with `--verify` (the
gathered frame must equal the whole frame rendered on one device, bit for
bit).  Started by tests/conftest.py before the test
process touches the GPU (no process that has initialised the GPU may exec
another program); tests/test_multirank_bench.py reads the result.

usage: python scripts/multirank_check.py <out.json>
"""
import json
import os
import pathlib
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]


def run(ranks: int, port: int) -> dict:
    env = dict(os.environ, BENCH_BACKEND="gloo", BENCH_SHARE_GPU="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", str(ranks),
           "--width", "320", "--height", "200", "--spp", "8", "--steps", "2", "--warmup", "2", "--verify",
           "--no-cpu-baseline"]
    t = time.time()
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    out = {"ranks": ranks, "rc": p.returncode, "seconds": round(time.time() - t, 1)}
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if lines:
        out["line"] = json.loads(lines[-1])
    if p.returncode != 0 or not lines:
        out["stderr"] = p.stderr[-3000:]
    return out


def run_single_process(ranks: int, extra) -> dict:
    """bench.py --gpus N with no launcher: one process, rt_multi over N
    "devices" that are all cuda:0 (BENCH_SHARE_GPU=1: peer copies, since RCCL
    refuses a repeated device)."""
    env = dict(os.environ, BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(ranks), "--verify", "--no-cpu-baseline", *extra]
    t = time.time()
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    out = {"ranks": ranks, "launcher": "none", "args": extra, "rc": p.returncode, "seconds": round(time.time() - t, 1)}
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if lines:
        out["line"] = json.loads(lines[-1])
    if p.returncode != 0 or not lines:
        out["stderr"] = p.stderr[-3000:]
    return out


def main():
    dst = pathlib.Path(sys.argv[1])
    res = []
    jobs = [lambda: run(2, 29611), lambda: run(3, 29612),
            lambda: run_single_process(3, ["--width", "320", "--height", "200", "--spp", "8", "--steps", "2",
                                           "--warmup", "2"]),
            lambda: run_single_process(8, ["--steps", "3", "--warmup", "3"])]  # the full C2 frame, 8 shares
    for job in jobs:
        try:
            res.append(job())
        except subprocess.TimeoutExpired:
            res.append({"rc": -1, "stderr": "timeout"})
        print(json.dumps(res[-1])[:400], flush=True)
        if res[-1]["rc"] != 0:
            break
    dst.write_text(json.dumps(res))


if __name__ == "__main__":
    main()
