"""How far the opt-in split-N order (reduce_kernel_splitn) lies from the reference's sequential
sum, per fp32 tensor, as a function of the client count — computed exactly on the CPU with the
oracle's restatement of both orders (oracle.c_reduce vs oracle.c_reduce_splitn, which the GPU
tests pin bit for bit to the kernels); --guard applies the kernel's cancellation guard (columns
whose terms nearly cancel take the sequential sum).  Drives the split-N selection limit (kSplitMaxN in
flearn_amd/csrc/fa_reduce.hip).  Test infrastructure / measurement only.

    python tests/splitn_error.py [--out profiles/r03/splitn_error.json]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import oracle  # noqa: E402
from flearn_amd import layouts  # noqa: E402


def tensors(layout):
    out, off = [], 0
    for k, shape, t in layout:
        if t != "f32":
            continue
        m = int(np.prod(shape, dtype=np.int64)) if shape else 1
        out.append((k, off, m))
        off += m
    return out, off


def data(kind, n, p, seed):
    x = oracle.fill_uniform(n, p, seed)  # U(-1,1), zero-mean across clients
    if kind == "near_common":  # clients trained from one global model: a shared value + 1% noise
        m = oracle.fill_uniform(1, p, seed + 1)
        x = (m + np.float32(0.01) * x).astype(np.float32)
    if kind == "cancelling":  # client pairs that nearly cancel: the mean is ~1e-4 of the values
        half = x[: (n + 1) // 2]
        y = np.empty_like(x)
        y[0::2] = half[: y[0::2].shape[0]]
        y[1::2] = -half[: y[1::2].shape[0]] + np.float32(1e-4) * oracle.fill_uniform(n // 2, p, seed + 7)
        x = y
    return x


def weights(kind, n, rng):
    if kind == "ones":
        return [1.0] * n
    if kind == "moon_int":  # MOONClient: agg_weight = len(trainloader), Python ints
        return [int(v) for v in rng.integers(1, 601, n)]
    return [float(v) for v in rng.uniform(0.5, 2.0, n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--ns", default="128,256,512,768,1024,1536,2048,3072,4096")
    ap.add_argument("--guard", action="store_true", help="with the kernel's cancellation guard")
    ap.add_argument("--data", default="zero_mean,near_common,cancelling")
    args = ap.parse_args()
    lay, p = tensors(layouts.get("lenet5"))
    rng = np.random.default_rng(0)
    rows = []
    for n in [int(v) for v in args.ns.split(",")]:
        for dk in args.data.split(","):
            for wk in ("ones", "moon_int", "float"):
                errs = []
                for seed in (1, 2, 3):
                    x = data(dk, n, p, seed + n)
                    w = weights(wk, n, rng)
                    w32 = np.asarray(w, np.float64).astype(np.float32)
                    denom = float(np.sum(w))
                    a = oracle.c_reduce(oracle.MODE_W32_DIV64, x, w32, denom)
                    b = oracle.c_reduce_splitn(oracle.MODE_W32_DIV64, x, w32, denom, guard=args.guard)
                    for k, off, m in lay:
                        ra, rb = a[off : off + m], b[off : off + m]
                        nrm = np.linalg.norm(ra)
                        errs.append(float(np.linalg.norm(ra - rb) / nrm) if nrm else 0.0)
                row = dict(n=n, data=dk, weights=wk, guard=args.guard, max_rel=max(errs),
                           median_rel=float(np.median(errs)))
                rows.append(row)
                print(json.dumps(row), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(rows, indent=1) + "\n")


if __name__ == "__main__":
    main()
