"""The C-ABI library loads here (no GPU) and exports exactly what include/flearn_amd.h declares;
argument validation fails with the documented codes before anything touches a device."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from flearn_amd import _native as na

HEADER = Path(__file__).resolve().parent.parent / "include" / "flearn_amd.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", text)))


def header_define(name):
    m = re.search(rf"#define\s+{name}\s+\(?(-?\d+)\)?", HEADER.read_text())
    return int(m.group(1))


@pytest.fixture(scope="module")
def L():
    return na.load()


def test_header_matches_binding_table():
    assert declared_functions() == sorted(na.EXPORTS)


def test_library_exports_every_declared_symbol(L):
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(na.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT\s+(fa_[a-z0-9_]+)$", out, flags=re.M))
    assert exported == set(declared_functions()), exported ^ set(declared_functions())


def test_abi_version_and_constants(L):
    assert L.fa_abi_version() == header_define("FA_ABI_VERSION") == na.ABI_VERSION
    assert header_define("FA_MODE_W32_DIV64") == na.MODE_W32_DIV64
    assert header_define("FA_MODE_W32_DIV32") == na.MODE_W32_DIV32
    assert header_define("FA_MODE_W64") == na.MODE_W64
    assert (header_define("FA_SRC_F64"), header_define("FA_SRC_I64"), header_define("FA_SRC_F32")) == (
        na.SRC_F64, na.SRC_I64, na.SRC_F32)
    for op, v in na.OP_BY_NAME.items():
        assert header_define(f"FA_OP_{op.upper()}") == v
    assert (header_define("FA_FENCE_RELEASE"), header_define("FA_FENCE_ACQUIRE")) == (na.FENCE_RELEASE,
                                                                                      na.FENCE_ACQUIRE)


def test_epilogue_struct_layout_matches_c(tmp_path):
    """ctypes' fa_epilogue must have the C compiler's size and field offsets."""
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stddef.h>\n#include <stdio.h>\n#include "flearn_amd.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(fa_epilogue),"
        "offsetof(fa_epilogue,op),offsetof(fa_epilogue,reserved),offsetof(fa_epilogue,prev),"
        "offsetof(fa_epilogue,v),offsetof(fa_epilogue,beta),offsetof(fa_epilogue,eta),"
        "offsetof(fa_epilogue,tau),offsetof(fa_epilogue,beta2),offsetof(fa_epilogue,h),"
        "offsetof(fa_epilogue,alpha),offsetof(fa_epilogue,n_clients),offsetof(fa_epilogue,v_out));return 0;}\n"
    )
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(HEADER.parent), str(src), "-o", str(exe)], check=True)
    c = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    E = na.Epilogue
    py = [ctypes.sizeof(E)] + [getattr(E, f).offset for f in ("op", "reserved", "prev", "v", "beta", "eta", "tau", "beta2",
                                                           "h", "alpha", "n_clients", "v_out")]
    assert c == py


FAKE = 0x100000  # never dereferenced: validation rejects the call first


def test_reduce_rejects_bad_arguments(L):
    rc = L.fa_reduce_f32(FAKE, 64, 0, 0, FAKE, 1.0, 0, 64, None, FAKE, None, None)
    assert rc == header_define("FA_ERR_ARG")
    assert b"n_clients" in L.fa_last_error()
    rc = L.fa_reduce_f32(None, 64, 2, 0, FAKE, 1.0, 0, 64, None, FAKE, None, None)
    assert rc == header_define("FA_ERR_ARG")
    rc = L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 64, None, None, None, None)
    assert rc == header_define("FA_ERR_ARG") and b"output" in L.fa_last_error()
    rc = L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 10, 60, None, FAKE, None, None)  # window > stride
    assert rc == header_define("FA_ERR_ARG")


def test_reduce_rejects_misaligned_windows(L):
    err_align = header_define("FA_ERR_ALIGN")
    assert L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 1, 8, None, FAKE, None, None) == err_align
    assert L.fa_reduce_f32(FAKE, 66, 2, 0, FAKE, 1.0, 0, 8, None, FAKE, None, None) == err_align
    assert L.fa_reduce_f32(FAKE + 4, 64, 2, 0, FAKE, 1.0, 0, 8, None, FAKE, None, None) == err_align
    assert L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 8, None, FAKE + 4, None, None) == err_align
    assert L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 8, None, None, FAKE + 8, None) == err_align


def test_unknown_mode_and_op(L):
    assert L.fa_reduce_f32(FAKE, 64, 2, 7, FAKE, 1.0, 0, 8, None, FAKE, None, None) == header_define("FA_ERR_ARG")
    epi = na.Epilogue(9, 0, FAKE, FAKE, 0.9, 0.1, 1e-9, 0.99)
    rc = L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 8, ctypes.byref(epi), FAKE, None, None)
    assert rc == header_define("FA_ERR_ARG")
    epi = na.Epilogue(na.OP_AVGM, 0, None, None, 0.9, 0.1, 1e-9, 0.99)  # op without state
    rc = L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 8, ctypes.byref(epi), FAKE, None, None)
    assert rc == header_define("FA_ERR_ARG")
    epi = na.Epilogue(na.OP_DYN, 0, None, FAKE, 0, 0, 0, 0, None, 0.01, 0)  # FedDyn without h
    rc = L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 8, ctypes.byref(epi), FAKE, None, None)
    assert rc == header_define("FA_ERR_ARG") and b"h" in L.fa_last_error()
    epi = na.Epilogue(na.OP_DYN, 0, None, FAKE, 0, 0, 0, 0, FAKE + 4, 0.01, 0)  # misaligned h
    rc = L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 8, ctypes.byref(epi), FAKE, None, None)
    assert rc == header_define("FA_ERR_ALIGN")
    epi = na.Epilogue(na.OP_DYN, 0, None, FAKE, 0, 0, 0, 0, FAKE, 0.01, 0)  # apply needs N
    rc = L.fa_opt_apply(na.PREC_F64, ctypes.byref(epi), None, FAKE, 8, None, FAKE, None)
    assert rc == header_define("FA_ERR_ARG")


def test_v_out_overlapping_v_is_refused(L):
    """v_out may not share a byte with v over the launch's columns (a shifted view would race the
    epilogue's loads); the exact alias was refused already."""
    for shift in (0, 4, 8 * 4):  # f64 elements: same address, half a quad later, 4 quads later
        epi = na.Epilogue(na.OP_AVGM, 0, FAKE, FAKE, 0.9, 0.1, 1e-9, 0.99, None, 0, 0, FAKE + 8 * shift)
        rc = L.fa_reduce_f32(FAKE, 4096, 2, 0, FAKE, 1.0, 0, 1024, ctypes.byref(epi), FAKE, None, None)
        assert rc == header_define("FA_ERR_ARG") and b"overlap" in L.fa_last_error() or shift == 0, shift
        assert rc == header_define("FA_ERR_ARG")
        rc = L.fa_opt_apply(na.PREC_F64, ctypes.byref(epi), FAKE, FAKE, 1024, None, FAKE, None)
        assert rc == header_define("FA_ERR_ARG")


def test_empty_window_is_a_no_op(L):
    assert L.fa_reduce_f32(FAKE, 64, 2, 0, FAKE, 1.0, 0, 0, None, FAKE, None, None) == 0
    assert L.fa_reduce_f64(FAKE, 64, 2, FAKE, 1.0, 0, 0, FAKE, None) == 0
    assert L.fa_reduce_i64(FAKE, 64, 2, FAKE, 1.0, 0, 0, FAKE, None) == 0


def test_apply_and_fill_validation(L):
    epi = na.Epilogue(na.OP_MEAN, 0, None, FAKE, 0.9, 0.1, 1e-9, 0.99)
    assert L.fa_opt_apply(na.PREC_F64, ctypes.byref(epi), FAKE, FAKE, 8, FAKE, None, None) == header_define("FA_ERR_ARG")
    assert L.fa_opt_apply(na.PREC_F64, None, FAKE, FAKE, 8, FAKE, None, None) == header_define("FA_ERR_ARG")
    assert L.fa_fill_uniform_f32(FAKE, 64, 70000, 64, 1, 0, 0, None) == header_define("FA_ERR_ARG")
    assert L.fa_fill_uniform_f32(FAKE, 8, 1, 64, 1, 0, 0, None) == header_define("FA_ERR_ARG")


def test_copy_validation(L):
    """fa_copy: 16-byte aligned pointers only (the caller then takes the copy engine), no
    negative sizes, and an empty copy touches nothing."""
    assert L.fa_copy(FAKE + 8, FAKE, 64, None) == header_define("FA_ERR_ALIGN")
    assert L.fa_copy(FAKE, FAKE + 4, 64, None) == header_define("FA_ERR_ALIGN")
    assert L.fa_copy(FAKE, FAKE, -1, None) == header_define("FA_ERR_ARG")
    assert L.fa_copy(None, FAKE, 64, None) == header_define("FA_ERR_ARG")
    assert L.fa_copy(None, None, 0, None) == 0


def test_push_and_ipc_validation(L):
    """fa_push: at most 8 destinations, 16-byte aligned pointers and size, no null destination;
    an empty push touches nothing.  fa_ipc_*: null arguments refused before any HIP call."""
    P = ctypes.c_void_p
    dsts = (P * 9)(*([FAKE] * 9))
    assert L.fa_push(FAKE, 64, dsts, 9, 0, None) == header_define("FA_ERR_ARG")
    assert L.fa_push(FAKE, 64, dsts, -1, 0, None) == header_define("FA_ERR_ARG")
    assert L.fa_push(FAKE, -16, dsts, 2, 0, None) == header_define("FA_ERR_ARG")
    assert L.fa_push(FAKE, 0, dsts, 2, 0, None) == 0
    assert L.fa_push(FAKE, 64, dsts, 0, 0, None) == 0
    assert L.fa_push(FAKE + 8, 64, dsts, 2, 0, None) == header_define("FA_ERR_ALIGN")
    assert L.fa_push(FAKE, 72, dsts, 2, 0, None) == header_define("FA_ERR_ALIGN")
    bad = (P * 2)(FAKE, None)
    assert L.fa_push(FAKE, 64, bad, 2, 0, None)
    assert L.fa_push(FAKE, 64, dsts, 2, -1, None) == header_define("FA_ERR_ARG") == header_define("FA_ERR_ARG")
    off = ctypes.c_int64()
    assert L.fa_ipc_handle(None, ctypes.create_string_buffer(64), ctypes.byref(off)) == header_define("FA_ERR_ARG")
    assert L.fa_ipc_open(None, ctypes.byref(P())) == header_define("FA_ERR_ARG")
    assert L.fa_ipc_close(None) == header_define("FA_ERR_ARG")
    assert header_define("FA_IPC_HANDLE_BYTES") == 64
    assert L.fa_copy_dma(FAKE, FAKE, -1, None) == header_define("FA_ERR_ARG")
    assert L.fa_copy_dma(None, FAKE, 64, None) == header_define("FA_ERR_ARG")
    assert L.fa_copy_dma(None, None, 0, None) == 0
    sts = (P * 9)(*([FAKE] * 9))
    assert L.fa_push_dma(FAKE, 64, dsts, 9, sts, None) == header_define("FA_ERR_ARG")
    assert L.fa_push_dma(FAKE, -1, dsts, 2, sts, None) == header_define("FA_ERR_ARG")
    assert L.fa_push_dma(FAKE, 0, dsts, 2, sts, None) == 0
    assert L.fa_push_dma(FAKE, 64, dsts, 2, None, None) == header_define("FA_ERR_ARG")
    assert L.fa_push_dma(FAKE, 64, bad, 2, sts, None) == header_define("FA_ERR_ARG")
    assert L.fa_stream_join(None, None, 0) == 0
    assert L.fa_stream_join(None, None, 2) == header_define("FA_ERR_ARG")
    assert L.fa_stream_join(None, sts, 17) == header_define("FA_ERR_ARG")


def test_piece_struct_layout_matches_c(tmp_path):
    src = tmp_path / "piece.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "flearn_amd.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu\\n", sizeof(fa_piece), offsetof(fa_piece,col),'
                   'offsetof(fa_piece,seg_off),offsetof(fa_piece,seg),offsetof(fa_piece,n_cols));return 0;}\n')
    exe = tmp_path / "piece"
    subprocess.run(["gcc", "-I", str(HEADER.parent), str(src), "-o", str(exe)], check=True)
    c = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    P = na.Piece
    assert c == [ctypes.sizeof(P), P.col.offset, P.seg_off.offset, P.seg.offset, P.n_cols.offset]


def _plan(L, cols, lens, op=0, grid=0):
    S = len(cols)
    c = (ctypes.c_int64 * max(S, 1))(*cols)
    n = (ctypes.c_int64 * max(S, 1))(*lens)
    cnt, g = ctypes.c_int64(-1), ctypes.c_int32(-1)
    assert L.fa_rows_plan(S, c, n, op, grid, None, 0, ctypes.byref(cnt), ctypes.byref(g)) == 0
    arr = (na.Piece * max(cnt.value, 1))()
    if cnt.value:
        small, g2 = ctypes.c_int64(), ctypes.c_int32()
        assert L.fa_rows_plan(S, c, n, op, grid, arr, cnt.value - 1, ctypes.byref(small),
                              ctypes.byref(g2)) == header_define("FA_ERR_SIZE")
    assert L.fa_rows_plan(S, c, n, op, grid, arr, cnt.value, ctypes.byref(cnt), ctypes.byref(g)) == 0
    return [(p.col, p.seg_off, p.seg, p.n_cols) for p in arr[: cnt.value]], g.value


@pytest.mark.parametrize("grid", [192, 7, 0])
def test_rows_plan_covers_every_segment_once(L, grid):
    """fa_rows_plan (host): pieces tile each segment exactly in equal 1-KiB-chunk multiples of at
    most 64 KiB of a row, stay inside one segment, come largest first; pieces[0].aux counts the
    leading wide pieces (> 2048 columns) the kernel sweeps in groups; the grid never exceeds the
    work items."""
    lens = [1, 3, 4, 63, 64, 255, 256, 257, 8191, 8192, 8193, 2_359_296, 0, 100_003]
    cols, c = [], 0
    for n in lens:
        cols.append(c)
        c += -(-max(n, 1) // 64) * 64
    ctypes_pieces = _plan_raw(L, cols, lens, grid)
    pieces, g = ctypes_pieces[0], ctypes_pieces[1]
    assert [p[3] for p in pieces] == sorted((p[3] for p in pieces), reverse=True)
    nwide = ctypes_pieces[2]
    assert nwide == sum(1 for p in pieces if p[3] > 2048)
    assert all(p[3] > 2048 for p in pieces[:nwide])
    claims = -(-nwide // 2) + (len(pieces) - nwide)
    assert 1 <= g <= claims and (grid == 0 or g == min(grid, claims))
    for s, (c0, n) in enumerate(zip(cols, lens)):
        mine = sorted((p for p in pieces if p[2] == s), key=lambda p: p[1])
        assert sum(p[3] for p in mine) == n
        off = 0
        for col, seg_off, _, w in mine:
            assert seg_off == off and col == c0 + off and 0 < w <= 16384 and seg_off % 256 == 0
            off += w
        if len(mine) > 1:  # equal cut: all but the last piece the same width
            assert len({p[3] for p in mine[:-1]}) == 1 and mine[-1][3] <= mine[0][3]


def _plan_raw(L, cols, lens, grid):
    S = len(cols)
    c = (ctypes.c_int64 * max(S, 1))(*cols)
    n = (ctypes.c_int64 * max(S, 1))(*lens)
    cnt, g = ctypes.c_int64(), ctypes.c_int32()
    assert L.fa_rows_plan(S, c, n, 0, grid, None, 0, ctypes.byref(cnt), ctypes.byref(g)) == 0
    arr = (na.Piece * max(cnt.value, 1))()
    assert L.fa_rows_plan(S, c, n, 0, grid, arr, cnt.value, ctypes.byref(cnt), ctypes.byref(g)) == 0
    return [(p.col, p.seg_off, p.seg, p.n_cols) for p in arr[: cnt.value]], g.value, (arr[0].aux if cnt.value else 0)


def test_rows_plan_empty(L):
    assert _plan(L, [0, 64], [0, 0]) == ([], 0)


def test_rows_entry_points_validate(L):
    cnt, g = ctypes.c_int64(), ctypes.c_int32()
    c = (ctypes.c_int64 * 1)(2)  # not 4-aligned
    n = (ctypes.c_int64 * 1)(8)
    assert L.fa_rows_plan(1, c, n, 0, 0, None, 0, ctypes.byref(cnt), ctypes.byref(g)) == header_define("FA_ERR_ARG")
    assert L.fa_rows_plan(1, c, n, 9, 0, None, 0, ctypes.byref(cnt), ctypes.byref(g)) == header_define("FA_ERR_ARG")
    err = header_define("FA_ERR_ARG")
    assert L.fa_reduce_f32_rows(FAKE, 0, 0, FAKE, 1.0, FAKE, 1, 1, FAKE, None, FAKE, None, None) == err
    assert L.fa_reduce_f32_rows(None, 2, 0, FAKE, 1.0, FAKE, 1, 1, FAKE, None, FAKE, None, None) == err
    assert L.fa_reduce_f32_rows(FAKE, 2, 0, FAKE, 1.0, FAKE, 1, 1, None, None, FAKE, None, None) == err  # work
    assert L.fa_reduce_f32_rows(FAKE, 2, 0, FAKE, 1.0, FAKE, 1, 1, FAKE, None, None, None, None) == err
    assert L.fa_reduce_f32_rows(FAKE, 2, 0, FAKE, 1.0, FAKE, 4, 5, FAKE, None, FAKE, None, None) == err  # grid
    assert L.fa_reduce_f32_rows(FAKE, 2, 0, FAKE, 1.0, FAKE, 1, 1, FAKE, None, FAKE + 4, None, None) == header_define("FA_ERR_ALIGN")
    assert L.fa_reduce_f32_rows(FAKE, 2, 0, FAKE, 1.0, FAKE, 0, 0, FAKE, None, FAKE, None, None) == 0  # no pieces
    assert L.fa_gather_rows(FAKE, 64, 2, 2, FAKE, FAKE, 1, None) == err  # element size
    assert L.fa_gather_rows(FAKE, 64, 0, 4, FAKE, FAKE, 1, None) == 0
    assert L.fa_gather_rows_f64(FAKE, 64, -1, FAKE, FAKE, 1, None) == err
    assert L.fa_gather_rows_f64(FAKE, -1, 2, FAKE, FAKE, 1, None) == err
    assert L.fa_gather_rows_f64(None, 64, 2, FAKE, FAKE, 1, None) == err
    assert L.fa_gather_rows_f64(FAKE, 64, 2, FAKE, FAKE, 0, None) == 0


def test_reduce_grid_knob(L):
    """fa_set_reduce_grid: process-wide, returns the previous value, refuses negatives."""
    assert L.fa_set_reduce_grid(0) == 0
    assert L.fa_set_reduce_grid(160) == 0
    assert L.fa_set_reduce_grid(224) == 160
    assert L.fa_set_reduce_grid(-1) == header_define("FA_ERR_ARG")
    assert L.fa_set_reduce_grid(0) == 224


def test_reduce_window_count(L):
    """fa_reduce_windows (host): how many launches fa_reduce_f32 makes — fused epilogues at
    >= 16 Mi columns in 3 windows, plain means of 8-16 Mi columns in 2, else 1 (DESIGN.md §4
    finding 26); one with a forced grid; unknown ops refused."""
    mean, avgm, adagrad = na.OP_MEAN, na.OP_AVGM, na.OP_ADAGRAD
    assert L.fa_reduce_windows(mean, 25_610_152) == 1  # NS
    assert L.fa_reduce_windows(mean, 11_699_112) == 2  # C2 / C4
    assert L.fa_reduce_windows(mean, 86_567_656) == 1
    assert L.fa_reduce_windows(mean, 44_426) == 1  # LeNet5
    assert L.fa_reduce_windows(avgm, 25_610_152) == 3  # C3
    assert L.fa_reduce_windows(adagrad, 86_567_656) == 3  # C5
    assert L.fa_reduce_windows(adagrad, (16 << 20) - 64) == 1
    assert L.fa_reduce_windows(na.OP_DYN, 16 << 20) == 3
    assert L.fa_reduce_windows(99, 1000) == header_define("FA_ERR_ARG")
    prev = L.fa_set_reduce_grid(128)
    try:
        assert L.fa_reduce_windows(adagrad, 86_567_656) == 1
    finally:
        L.fa_set_reduce_grid(prev)


def test_cache_fence_rejects_an_unknown_kind(L):
    assert L.fa_cache_fence(7, None) == header_define("FA_ERR_ARG")
    assert b"fence" in L.fa_last_error()
