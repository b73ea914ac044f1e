"""Diagnose the push gather's stale IPC imports: the export -> map -> unmap ->
free -> re-export sequence of flearn_amd.dist, repeated, with every handle, exported range and
mapping logged.

    python tools/ipc_probe.py --world 3 --iters 40 --alloc torch --after-unmap none --free del \
        --sizes vary --out gpurun_out/ipc/torch_none_del

`world` fresh processes share cuda:0 over gloo (as tests/test_gpu_multirank.py does).  Each
iteration, on every rank: allocate a bucket (torch's caching allocator, or fa_dev_alloc: an
allocation of its own), stamp a token (rank, iteration, magic, random) into its first 16 bytes,
export it (fa_ipc_handle: the handle of the allocation holding the bucket and the bucket's
offset in it; fa_mem_range: that allocation's base and size), exchange (all_gather_object),
map every peer's (fa_ipc_open), read the 16 bytes through each mapping (fa_copy_dma), barrier,
unmap, optionally barrier again, free (del; + empty_cache; or fa_dev_free).  A mapping whose
bytes are not the peer's current token is STALE; the token it did hold names the iteration
whose bucket the import really mapped.  Per rank a JSON log; rank 0 prints the summary.
Test and diagnosis infrastructure; not the product path.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

MAGIC = 0x5A17C0DE  # fits int32


def rank_main(rank, world, port, args):
    import numpy as np
    import torch
    import torch.distributed as dist

    from flearn_amd import _native as na
    from flearn_amd import dist as fd

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    L = na.lib()
    rng = np.random.default_rng(1000 + rank)
    probe = torch.empty(4, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    seen = {}  # handle bytes -> first iteration
    log = []
    keep = []
    try:
        for it in range(args.iters):
            # every local step guarded, every collective always reached: one rank's failure is
            # recorded, never a desynchronised collective
            cols = args.cols + (it % 5) * 65536 if args.sizes == "vary" else args.cols
            rec = {"it": it, "cols": cols, "peers": {}}
            own = buf = None
            mine = None
            try:
                if args.alloc == "own" and args.free == "reuse":
                    if len(keep) < 3:
                        keep.append(fd.DeviceBuffer(cols * 4, dev))
                    buf = keep[it % 3].tensor(torch.float32)
                elif args.alloc == "own":
                    own = fd.DeviceBuffer(cols * 4, dev)
                    buf = own.tensor(torch.float32)
                    if args.free == "keep":
                        keep.append(own)
                        own = None
                else:
                    buf = torch.empty(cols, dtype=torch.float32, device=dev)
                    if args.neighbours:  # other tensors sharing (and recycling) the segment
                        keep.append(torch.empty(int(rng.integers(1, 4)) * 65536, dtype=torch.float32, device=dev))
                        if len(keep) > 3:
                            keep.pop(0)
                tok = [rank, it, MAGIC, int(rng.integers(-2**31, 2**31 - 1))]
                buf.view(torch.int32)[:4].copy_(torch.tensor(tok, dtype=torch.int32))
                torch.cuda.synchronize(dev)
                h, off = ctypes.create_string_buffer(64), ctypes.c_int64(0)
                base, size = ctypes.c_void_p(), ctypes.c_int64(0)
                rc_r = L.fa_mem_range(buf.data_ptr(), ctypes.byref(base), ctypes.byref(size))
                rc_h = L.fa_ipc_handle(buf.data_ptr(), h, ctypes.byref(off))
                hb = bytes(h.raw)
                rec.update(ptr=hex(buf.data_ptr()), base=hex(base.value or 0), size=int(size.value),
                           offset=int(off.value), handle=hb.hex(), handle_seen_at=seen.get(hb))
                if rc_r or rc_h:  # e.g. hipIpcGetMemHandle refusing a re-allocated address
                    rec["export_error"] = L.fa_last_error().decode(errors="replace")
                else:
                    seen.setdefault(hb, it)
                    mine = (hb, int(off.value), tok)
            except Exception as e:  # noqa: BLE001
                rec["local_error"] = f"{type(e).__name__}: {e}"
            infos = [None] * world
            dist.all_gather_object(infos, mine)
            opened = []
            for r, info in enumerate(infos):
                if r == rank or info is None:
                    continue
                phb, poff, ptok = info
                try:
                    pb = ctypes.c_void_p()
                    rc = L.fa_ipc_open(phb, ctypes.byref(pb))
                    if rc != 0 or not pb.value:
                        rec["peers"][r] = {"open_error": L.fa_last_error().decode(errors="replace")}
                        continue
                    opened.append(pb.value)
                    na.check(L.fa_copy_dma(probe.data_ptr(), pb.value + poff, 16, stream.cuda_stream), "fa_copy_dma")
                    stream.synchronize()
                    got = probe.tolist()
                    ent = {"mapped": hex(pb.value), "ok": got == ptok}
                    if got != ptok:
                        ent["read"] = got
                        if got[2] == MAGIC:
                            ent["stale_holds"] = {"rank": got[0], "iteration": got[1]}
                    rec["peers"][r] = ent
                except Exception as e:  # noqa: BLE001
                    rec["peers"][r] = {"error": f"{type(e).__name__}: {e}"}
            dist.barrier()
            for b in opened:
                if L.fa_ipc_close(b) != 0:
                    rec.setdefault("close_errors", []).append(L.fa_last_error().decode(errors="replace"))
            if args.after_unmap == "barrier":
                dist.barrier()
            try:
                del buf
                if own is not None:
                    own.free()
                    own = None
                elif args.free == "empty":
                    torch.cuda.empty_cache()
            except Exception as e:  # noqa: BLE001
                rec["free_error"] = f"{type(e).__name__}: {e}"
            log.append(rec)
        torch.cuda.synchronize(dev)
        dist.barrier()
    finally:
        Path(args.out).mkdir(parents=True, exist_ok=True)
        (Path(args.out) / f"rank{rank}.json").write_text(json.dumps(log, indent=1))
        stale = {"stale_or_failed_mappings": sum(1 for rec in log for p in rec["peers"].values() if not p.get("ok")),
                 "export_errors": sum(1 for rec in log if "export_error" in rec),
                 "local_errors": sum(1 for rec in log if "local_error" in rec or "free_error" in rec),
                 "iterations": len(log)}
        allr = [None] * world
        try:
            dist.all_gather_object(allr, stale)
        except Exception:  # noqa: BLE001 - the summary is best effort
            pass
        if rank == 0:
            print(json.dumps({"variant": vars(args), "per_rank": allr}), flush=True)
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--cols", type=int, default=700_032)
    ap.add_argument("--alloc", choices=("torch", "own"), default="torch")
    ap.add_argument("--after-unmap", choices=("none", "barrier"), default="none")
    ap.add_argument("--free", choices=("del", "empty", "keep", "reuse"), default="del",
                    help="keep (own): a new bucket each iteration, none ever freed; reuse (own): 3 buckets "
                         "allocated once, iteration i re-exports bucket i %% 3 (the receive pool's pattern).  "
                         "(The r05c 'retire' variants — hipFree, then the freed range reserved with "
                         "hipMemAddressReserve — ran on commit 10346de's fa_dev_retire, since removed)")
    ap.add_argument("--sizes", choices=("fixed", "vary"), default="vary")
    ap.add_argument("--neighbours", action="store_true", help="torch: other tensors share the segments")
    ap.add_argument("--out", default="gpurun_out/ipc/probe")
    args = ap.parse_args()
    import socket

    import torch.multiprocessing as mp

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    t0 = time.time()
    mp.start_processes(rank_main, args=(args.world, port, args), nprocs=args.world, join=True, start_method="spawn")
    print(f"# {time.time() - t0:.1f} s", file=sys.stderr)


if __name__ == "__main__":
    main()
