"""fa_copy (the kernel copy that stores Strategy.server's result straight into pinned host
memory, bucket.Packer._unpack_zero_copy) and the host-upload pipeline around it on the GPU:
byte-exact for every direction and for sizes that end in a partial 16-byte quad, and the
zero-copy unpack equal to the staged one."""
import numpy as np
import pytest
import torch

from flearn_amd import _native as na

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [16, 4096, 1 << 20, (1 << 20) + 4, (3 << 20) + 13, 123_456_789])
@pytest.mark.parametrize("direction", ["d2h", "h2d", "d2d"])
def test_copy_is_byte_exact(nbytes, direction, cuda):
    L = na.lib()
    src_bytes = torch.randint(0, 256, (nbytes + 16,), dtype=torch.uint8)
    if direction == "h2d":
        src = src_bytes.pin_memory()
        dst = torch.full((nbytes + 16,), 7, dtype=torch.uint8, device="cuda")
    else:
        src = src_bytes.to("cuda")
        dst = (torch.full((nbytes + 16,), 7, dtype=torch.uint8).pin_memory() if direction == "d2h"
               else torch.full((nbytes + 16,), 7, dtype=torch.uint8, device="cuda"))
    s = torch.cuda.current_stream()
    na.check(L.fa_copy(dst.data_ptr(), src.data_ptr(), nbytes, s.cuda_stream), "fa_copy")
    s.synchronize()
    got = dst.cpu()
    assert torch.equal(got[:nbytes], src_bytes[:nbytes])
    assert (got[nbytes:] == 7).all()  # nothing past the end


def test_zero_copy_unpack_equals_staged(cuda):
    """The same server round returned through both unpack paths: bit-equal values, and the
    zero-copy values are fresh per call (not overwritten by the next round)."""
    import flearn_amd
    from flearn_amd import layouts

    lay = layouts.get("resnet18")
    p = layouts.fp32_elems(lay)
    rng = np.random.default_rng(5)
    ups = []
    for i in range(6):
        sd = layouts.synthetic_state_dict(lay, rng.standard_normal(p).astype(np.float32), counter=i + 1)
        ups.append({"params": sd, "agg_weight": float(i + 1)})
    s = flearn_amd.AVG()
    out = {}
    for zc in (True, False):
        s.engine.packer.zero_copy_out = zc
        out[zc] = s.server(ups, 0)["w_glob"]
        assert s.engine.packer.last_pack_paths["f32"] == "async"
    for k in out[False]:
        a, b = out[True][k], out[False][k]
        assert type(a) is type(b) and np.asarray(a).dtype == np.asarray(b).dtype
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), k
    s.engine.packer.zero_copy_out = True
    first = {k: np.array(v, copy=True) for k, v in out[True].items()}
    s.server(ups[::-1], 0)
    for k in first:
        assert np.asarray(out[True][k]).tobytes() == first[k].tobytes(), k


def test_async_pack_falls_back_for_values_off_the_plan(cuda):
    """One upload value the native pack refuses (a non-contiguous array): that upload's chunk is
    packed from Python instead (the others stay native), with the same result."""
    import flearn_amd
    from flearn_amd import layouts

    lay = layouts.get("resnet18")
    p = layouts.fp32_elems(lay)
    rng = np.random.default_rng(9)
    ups = [{"params": layouts.synthetic_state_dict(lay, rng.standard_normal(p).astype(np.float32), counter=1),
            "agg_weight": 1.0 + i} for i in range(5)]
    s = flearn_amd.AVG()
    a = s.server(ups, 0)["w_glob"]
    assert s.engine.packer.last_pack_paths["f32"] == "async"
    k = next(k for k, v in ups[2]["params"].items() if v.ndim == 4)
    v = ups[2]["params"][k]
    ups[2]["params"][k] = np.asfortranarray(v)  # same values, not C-contiguous
    b = s.server(ups, 0)["w_glob"]
    assert s.engine.packer.last_pack_paths["f32"] == "mixed"
    for key in a:
        assert np.asarray(a[key]).tobytes() == np.asarray(b[key]).tobytes(), key


@pytest.mark.parametrize("n_dsts", [1, 2, 3, 8])
@pytest.mark.parametrize("grid", [0, 1, 7, 64, 1024])
def test_push_copies_every_destination(n_dsts, grid, cuda):
    """fa_push (the one-shot all-gather's store kernel) into local buffers: every destination
    gets the source, byte for byte, for sizes that are not a multiple of the grid's span, and
    nothing past the end is touched."""
    import ctypes

    L = na.lib()
    for nq in (1, 255, 256, 4097, 58_336, 200_003):
        nbytes = nq * 16
        src = torch.randint(0, 2**31 - 1, (nq * 4,), dtype=torch.int32, device="cuda")
        dsts = [torch.full((nq * 4 + 64,), -5, dtype=torch.int32, device="cuda") for _ in range(n_dsts)]
        ptrs = (ctypes.c_void_p * n_dsts)(*[d.data_ptr() for d in dsts])
        s = torch.cuda.current_stream()
        na.check(L.fa_push(src.data_ptr(), nbytes, ptrs, n_dsts, grid, s.cuda_stream), "fa_push")
        s.synchronize()
        for d in dsts:
            assert torch.equal(d[: nq * 4], src), (n_dsts, grid, nq)
            assert (d[nq * 4 :] == -5).all()
