"""Rehearsal of bench.py's multi-rank path on ONE GPU (every rank on cuda:0,
gloo instead of RCCL, which refuses two ranks on one device): torchrun with 2
and 3 ranks, `--verify` (rank 0 re-renders the frame alone and compares the
gathered frame bit for bit).  Started by tests/conftest.py before the test
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


def main():
    dst = pathlib.Path(sys.argv[1])
    res = []
    for ranks, port in ((2, 29611), (3, 29612)):
        try:
            res.append(run(ranks, port))
        except subprocess.TimeoutExpired:
            res.append({"ranks": ranks, "rc": -1, "stderr": "timeout"})
        print(json.dumps(res[-1])[:400], flush=True)
        if res[-1]["rc"] != 0:
            break
    dst.write_text(json.dumps(res))


if __name__ == "__main__":
    main()
