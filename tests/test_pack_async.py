"""The native async pack behind the client-side update's zero-copy chunks
(csrc/fa_pyhost.c fa_py_pack_start / fa_pack_wait / fa_py_pack_end, strategy/_update.py
_AsyncPack): every chunk's bytes land where the Python pack puts them, values off the plan
fall back with nothing copied, and concurrent packs from several threads stay separate."""
import threading

import numpy as np
import pytest
import torch

from flearn_amd.strategy._update import _AsyncPack


def _plan(shapes, per_chunk):
    """(chunks, total): layout entries (key, shape, offset, numel) in chunks of per_chunk keys,
    64-element aligned like DeviceUpdater._layout."""
    lay, off = [], 0
    for i, s in enumerate(shapes):
        n = int(np.prod(s)) if s else 1
        lay.append((f"k{i}", s, off, n))
        off += -(-max(n, 1) // 64) * 64
    groups = [lay[i : i + per_chunk] for i in range(0, len(lay), per_chunk)]
    chunks = [(g[0][2], None, None, None, g) for g in groups]
    return chunks, off


def _dicts(shapes, gdt, seed):
    rng = np.random.default_rng(seed)
    local = {f"k{i}": rng.standard_normal(s).astype(np.float32) for i, s in enumerate(shapes)}
    glob = {f"k{i}": rng.standard_normal(s).astype(gdt) for i, s in enumerate(shapes)}
    return local, glob


SHAPES = [(64, 3, 7, 7), (64,), (), (1000, 1000), (3,), (0,), (257, 129), (2048, 512), (5,)]


@pytest.mark.parametrize("gdt,with_local,per_chunk", [(np.float64, True, 2), (np.float32, True, 4),
                                                      (np.float64, False, 1), (np.float64, True, 100)])
def test_chunks_land_like_the_python_pack(gdt, with_local, per_chunk):

    chunks, total = _plan(SHAPES, per_chunk)
    lh = np.full(total, -1, np.float32)
    gh = np.full(total, -1, gdt)
    ap = _AsyncPack(chunks, lh.ctypes.data if with_local else None, gh.ctypes.data, torch.from_numpy(gh).dtype)
    for seed in range(3):  # the plan is reused across calls
        local, glob = _dicts(SHAPES, gdt, seed)
        h = ap.start(local if with_local else None, glob)
        assert h is not None
        for j, (_f, _e, _pl, _pg, g) in enumerate(chunks):
            ap.wait(h, j)
            for k, s, o, n in g:  # chunk j is complete as soon as its wait returns
                assert np.array_equal(gh[o : o + n], glob[k].reshape(-1))
                if with_local:
                    assert np.array_equal(lh[o : o + n], local[k].reshape(-1))
        ap.end(h)
    if not with_local:
        assert (lh == -1).all()


def test_end_without_waits_finishes_every_copy():
    chunks, total = _plan(SHAPES * 4, 3)
    shapes = SHAPES * 4
    lh, gh = np.zeros(total, np.float32), np.zeros(total)
    ap = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
    local, glob = _dicts(shapes, np.float64, 7)
    h = ap.start(local, glob)
    ap.end(h)
    for _f, _e, _pl, _pg, g in chunks:
        for k, s, o, n in g:
            assert np.array_equal(gh[o : o + n], glob[k].reshape(-1))
            assert np.array_equal(lh[o : o + n], local[k].reshape(-1))


@pytest.mark.parametrize("fault", ["dtype", "missing", "shape", "noncontig", "tensor", "dict_subclass"])
def test_values_off_the_plan_fall_back_with_nothing_copied(fault):
    chunks, total = _plan(SHAPES, 2)
    lh, gh = np.zeros(total, np.float32), np.zeros(total)
    ap = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
    local, glob = _dicts(SHAPES, np.float64, 1)
    k = "k6"
    if fault == "dtype":
        glob[k] = glob[k].astype(np.float32)
    elif fault == "missing":
        del local[k]
    elif fault == "shape":
        glob[k] = glob[k][:-1]
    elif fault == "noncontig":
        local[k] = np.asfortranarray(local[k])
    elif fault == "tensor":
        glob[k] = torch.from_numpy(glob[k])
    else:  # a dict subclass may override item lookup: the native pack does not read it

        class D(dict):
            def __getitem__(self, key):
                return super().__getitem__(key) * 0

        local = D(local)
    assert ap.start(local, glob) is None
    assert not lh.any() and not gh.any()


def test_concurrent_packs_from_threads():
    shapes = [(300_000,), (7,), (123_457,), (64, 64)] * 3
    chunks, total = _plan(shapes, 2)
    errors = []

    def run(seed):
        try:
            lh, gh = np.zeros(total, np.float32), np.zeros(total)
            ap = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
            for r in range(20):
                local, glob = _dicts(shapes, np.float64, seed * 100 + r)
                h = ap.start(local, glob)
                for j in range(len(chunks)):
                    ap.wait(h, j)
                ap.end(h)
                for _f, _e, _pl, _pg, g in chunks:
                    for k, s, o, n in g:
                        assert np.array_equal(gh[o : o + n], glob[k].reshape(-1))
                        assert np.array_equal(lh[o : o + n], local[k].reshape(-1))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_values_stay_alive_until_end():
    """The pack holds its own references: the caller may drop the dicts right after start."""
    chunks, total = _plan([(1 << 20,)] * 6, 1)
    lh, gh = np.zeros(total, np.float32), np.zeros(total)
    ap = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
    local, glob = _dicts([(1 << 20,)] * 6, np.float64, 3)
    expect_l = {k: v.copy() for k, v in local.items()}
    expect_g = {k: v.copy() for k, v in glob.items()}
    h = ap.start(local, glob)
    del local, glob
    ap.end(h)
    for _f, _e, _pl, _pg, g in chunks:
        for k, s, o, n in g:
            assert np.array_equal(gh[o : o + n], expect_g[k]) and np.array_equal(lh[o : o + n], expect_l[k])


def test_bad_wait_index_raises():
    chunks, total = _plan(SHAPES, 2)
    lh, gh = np.zeros(total, np.float32), np.zeros(total)
    ap = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
    h = ap.start(*_dicts(SHAPES, np.float64, 0))
    with pytest.raises(RuntimeError):
        ap.wait(h, len(chunks))
    ap.end(h)


@pytest.mark.parametrize("threads", [1, 2])
def test_worker_cap_still_copies_everything(threads):
    from flearn_amd.bucket import AsyncPack

    shapes = [(200_000,), (3,), (70_001,)] * 4
    chunks, total = _plan(shapes, 3)
    lh, gh = np.zeros(total, np.float32), np.zeros(total)
    base = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
    ap = AsyncPack(base.keys, base.desc.reshape(7, -1).T.copy(), base.nchunks, threads=threads)
    local, glob = _dicts(shapes, np.float64, 4)
    h = ap.start((local, glob))
    for j in range(ap.nchunks):
        ap.wait(h, j)
    ap.end(h)
    for _f, _e, _pl, _pg, g in chunks:
        for k, s, o, n in g:
            assert np.array_equal(gh[o : o + n], glob[k].reshape(-1)) and np.array_equal(lh[o : o + n], local[k].reshape(-1))


@pytest.mark.parametrize("ndev,n,wire", [(1, 7, ()), (2, 5, ()), (3, 9, (0, 4, 8)), (1, 30, (3,))])
def test_server_row_chunks_land_like_the_python_pack(ndev, n, wire):
    """Packer._async_rows (the loopback server's native pack): every packed row's pieces land at
    the bucket layout's offsets of its shard's staging row — checked on CPU staging against the
    values themselves — chunk bounds grow 1, 2, 4, ... and cover every row once, and rows the
    wire codec already holds (here: marked) are skipped."""
    from flearn_amd.bucket import Packer, make_plan
    from flearn_amd.semantics import KIND_F32

    rng = np.random.default_rng(n)
    shapes = {"a": (300, 7), "b": (5,), "c": (64, 64), "d": (3, 3, 3, 11), "e": (1,)}
    ups = [{k: rng.standard_normal(s).astype(np.float32) for k, s in shapes.items()} for _ in range(n)]
    plan = make_plan([1.0] * n, ups)
    packer = Packer([torch.device("cpu")] * ndev)
    g = plan.groups[KIND_F32]
    shards = packer.shards(plan, KIND_F32)
    assert len(shards) == ndev
    pieces = packer._pieces(g, shards)
    hosts = [torch.full((n, sh.width), -7.0) for sh in shards]
    rows = [object() if r in wire else None for r in range(n)]
    aps, bounds = packer._async_rows(plan, pieces, hosts, rows)
    assert bounds[0] == (0, 1) and bounds[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    sizes = [hi - lo for lo, hi in bounds]
    cap = max(1, -(-n // 12))
    assert sizes[0] == 1 and max(sizes) <= cap and all(b >= a for a, b in zip(sizes[:-1], sizes[1:-1]))
    for j, ap in enumerate(aps):
        h = ap.start(ups)
        assert h is not None
        ap.wait(h, 0)
        ap.end(h)
    for r in range(n):
        for s, a, b, sh, d in pieces:
            got = hosts[sh.index][r, d : d + (b - a)].numpy()
            if r in wire:
                assert (got == -7.0).all()
            else:
                assert np.array_equal(got, ups[r][s.key].reshape(-1)[a:b]), (r, s.key, sh.index)


def test_ordered_dicts_are_packed():
    import collections

    chunks, total = _plan(SHAPES, 3)
    lh, gh = np.zeros(total, np.float32), np.zeros(total)
    ap = _AsyncPack(chunks, lh.ctypes.data, gh.ctypes.data, torch.float64)
    local, glob = _dicts(SHAPES, np.float64, 11)
    h = ap.start(collections.OrderedDict(local), collections.OrderedDict(glob))
    assert h is not None
    ap.end(h)
    for _f, _e, _pl, _pg, g in chunks:
        for k, s, o, n in g:
            assert np.array_equal(gh[o : o + n], glob[k].reshape(-1)) and np.array_equal(lh[o : o + n], local[k].reshape(-1))
