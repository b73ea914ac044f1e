"""Host (no GPU): property tests of the wire codec (flearn_amd/wire.py over csrc/fa_wire.cpp)
against the reference's Encrypt (Encrypt.py:17-44 = base64(pickle)): for arbitrary upload-like
objects — nested dicts / OrderedDicts / lists / tuples of numpy arrays of several dtypes, byte
orders, memory orders and shapes (0-d and empty included), numpy and Python scalars, strings and
bytes — encode() emits exactly base64.b64encode(pickle.dumps(obj)) and decode() returns what
pickle.loads returns, through both the scanner / pinned-row route and the small-upload route."""
import base64
import collections
import pickle

import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from flearn_amd import wire
from test_wire import same

DTYPES = ["<f4", "<f4", "<f8", ">f8", "<i8", "<f2", "|b1", "|u1", "<i4", ">f4"]


@st.composite
def arrays(draw):
    dt = np.dtype(draw(st.sampled_from(DTYPES)))
    shape = tuple(draw(st.lists(st.integers(0, 9), min_size=0, max_size=3)))
    n = int(np.prod(shape, dtype=np.int64))
    raw = draw(st.binary(min_size=n * dt.itemsize, max_size=n * dt.itemsize))
    a = np.frombuffer(raw, dtype=dt).reshape(shape).copy()
    if draw(st.booleans()) and a.ndim > 1:
        a = np.asfortranarray(a)
    return a


leaf = st.one_of(arrays(), arrays(), st.floats(allow_nan=False), st.integers(-2**40, 2**40),
                 st.text(max_size=8), st.binary(max_size=8), st.none(), st.booleans(),
                 st.floats(allow_nan=False).map(np.float64), st.integers(0, 100).map(np.int64))
keys = st.text(min_size=1, max_size=6)
tree = st.recursive(
    leaf,
    lambda ch: st.one_of(st.dictionaries(keys, ch, max_size=4),
                         st.dictionaries(keys, ch, max_size=4).map(collections.OrderedDict),
                         st.lists(ch, max_size=3), st.lists(ch, max_size=3).map(tuple)),
    max_leaves=12)
upload = st.builds(lambda w, p: {"agg_weight": w, "params": p},
                   st.one_of(st.floats(0.0, 1e3, allow_nan=False), st.integers(1, 600)),
                   st.dictionaries(keys, arrays(), min_size=1, max_size=6))


@settings(max_examples=120, deadline=None)
@given(st.one_of(upload, tree))
def test_encode_is_reference_and_decode_round_trips(obj):
    ref_text = base64.b64encode(pickle.dumps(obj)).decode()
    assert wire.Encrypt().encode(obj) == ref_text
    want = pickle.loads(pickle.dumps(obj))
    same(wire.Encrypt(fast_min_chars=0).decode(ref_text), want, "scanner route")
    same(wire.Encrypt().decode(ref_text), want, "default route")
