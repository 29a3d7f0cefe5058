"""The MPI-compatible wire frame: the engine's
pastar_wire_* entry points against the reference's own lz4sup.cpp
(pastar_lz4_en / pastar_lz4_dec, lz4sup.cpp:13-70).

- frames byte-identical to the committed fixtures, which the reference's
  pastar_lz4_en made (tests/golden/make_wire_fixtures.py);
- where oracle/_ref/libref_lz4sup.so is built (this container: the
  reference's lz4sup.cpp compiled in place against liblz4 1.9.3), the same
  on fresh random inputs, and each side decodes the other's frames;
- the decoder rejects truncated and corrupt frames without reading or
  writing out of bounds;
- node records in Node<N>::serialize field order (Node.h:57-64).
Host code only: no GPU.
"""
import ctypes
import hashlib
import importlib.util
import json
import os
import random
import struct

import pytest

from mpi_pastar_msa_amd import _native as nat

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "wire_lz4.json")
REF_LIB = os.path.join(HERE, "..", "oracle", "_ref", "libref_lz4sup.so")

_spec = importlib.util.spec_from_file_location("make_wire_fixtures", os.path.join(HERE, "golden", "make_wire_fixtures.py"))
fixtures = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(fixtures)


def encode(data):
    L = nat.lib()
    bound = ctypes.c_int64()
    assert L.pastar_wire_frame_bound(len(data), ctypes.byref(bound)) == 0
    out = ctypes.create_string_buffer(bound.value)
    n = ctypes.c_int64()
    src = ctypes.create_string_buffer(data, max(1, len(data)))
    assert L.pastar_wire_frame_encode(src, len(data), out, bound.value, ctypes.byref(n)) == 0
    assert n.value <= bound.value
    return out.raw[:n.value]


def decode(frame, cap=None):
    """(status, bytes incl. the trailing NUL)"""
    L = nat.lib()
    orig = struct.unpack_from("<I", frame, 8)[0] if len(frame) >= 12 else 0
    cap = orig if cap is None else cap
    out = ctypes.create_string_buffer(max(1, cap))
    n = ctypes.c_int64(-1)
    src = ctypes.create_string_buffer(frame, max(1, len(frame)))
    rc = L.pastar_wire_frame_decode(src, len(frame), out, cap, ctypes.byref(n))
    return rc, (out.raw[:n.value] if rc == 0 else None)


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as fh:
        return json.load(fh)["cases"]


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_LIB):
        pytest.skip("oracle/_ref/libref_lz4sup.so not built (no /root/reference or liblz4 here)")
    lib = ctypes.CDLL(REF_LIB)
    return lib


def ref_decode(lib, frame):
    orig = struct.unpack_from("<I", frame, 8)[0]
    bound = struct.unpack_from("<I", frame, 4)[0]
    out = ctypes.create_string_buffer(max(bound, orig))
    n = lib.ref_lz4_dec(frame, len(frame), out, len(out))
    assert n == orig
    return out.raw[:n]


def test_frames_match_reference_fixtures(golden):
    assert len(golden) >= 30
    for c in golden:
        data = fixtures.make_case(c["kind"], c["size"], c["seed"])
        f = encode(data)
        assert len(f) == c["frame_len"], (c["kind"], c["size"])
        if "frame_hex" in c:
            assert f.hex() == c["frame_hex"], (c["kind"], c["size"])
        assert hashlib.sha256(f).hexdigest() == c["sha256"], (c["kind"], c["size"])
        total, bound, orig = struct.unpack_from("<III", f)
        assert total == len(f) and orig == len(data) + 1 and bound == orig + orig // 255 + 16
        rc, back = decode(f)
        assert rc == 0 and back == data + b"\0"


def test_frames_match_reference_library_random(ref):
    rng = random.Random(20261017)
    kinds = ["random", "text", "runs", "nodes4", "nodes8", "mixed"]
    for i in range(120):
        kind = rng.choice(kinds)
        size = rng.choice((rng.randrange(0, 40), rng.randrange(40, 5000), rng.randrange(60000, 70000),
                           rng.randrange(100, 400) if kind.startswith("nodes") else rng.randrange(5000, 150000)))
        data = fixtures.make_case(kind, size, 1000 + i)
        mine = encode(data)
        theirs = fixtures.ref_frame(ref, data)
        assert mine == theirs, (kind, size)
        assert ref_decode(ref, mine) == data + b"\0"


def test_decode_reference_frames(ref):
    for i, size in enumerate((1, 13, 500, 65547, 123456)):
        data = fixtures.make_case("mixed", size, 77 + i)
        rc, back = decode(fixtures.ref_frame(ref, data))
        assert rc == 0 and back == data + b"\0"


def test_decoder_rejects_bad_frames():
    data = fixtures.make_case("mixed", 3000, 9)
    f = encode(data)
    assert decode(f)[0] == 0
    # truncated: the header's total exceeds the frame
    assert decode(f[:-1])[0] != 0
    assert decode(f[:11])[0] != 0
    # output larger than the caller's buffer
    assert decode(f, cap=len(data))[0] != 0
    # every single-byte corruption of the block either decodes to exactly
    # orig bytes or is rejected; none may crash
    rng = random.Random(5)
    for _ in range(400):
        b = bytearray(f)
        at = rng.randrange(12, len(b))
        b[at] ^= 1 << rng.randrange(8)
        rc, back = decode(bytes(b))
        assert rc != 0 or len(back) == len(data) + 1
    # an offset reaching before the output start
    bad = struct.pack("<III", 12 + 8, 32, 9) + bytes([0x10, ord("a"), 0x20, 0x00, 0x40]) + b"\0\0\0"
    assert decode(bad[:12 + 5])[0] != 0


def test_bound_and_argument_errors():
    L = nat.lib()
    b = ctypes.c_int64()
    assert L.pastar_wire_frame_bound(0, ctypes.byref(b)) == 0 and b.value == 12 + 1 + 16
    assert L.pastar_wire_frame_bound(-1, ctypes.byref(b)) < 0
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_int64()
    assert L.pastar_wire_frame_encode(b"abcdef", 6, out, 10, ctypes.byref(n)) < 0  # capacity below the bound


def _nodes(n, count, seed):
    rng = random.Random(seed)
    arr = (nat.pastar_node * count)()
    for i in range(count):
        for k in range(n):
            arr[i].pos[k] = rng.randrange(0, 65536)
        arr[i].g = rng.randrange(-2**31, 2**31)
        arr[i].f = rng.randrange(-2**31, 2**31)
        arr[i].parent_mask = rng.randrange(1, 1 << n)
    return arr


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_node_records_pack_in_serialize_order(n):
    L = nat.lib()
    count = 37
    arr = _nodes(n, count, n)
    rec = 12 + 2 * n
    buf = ctypes.create_string_buffer(rec * count)
    ln = ctypes.c_int64()
    assert L.pastar_wire_pack_nodes(arr, count, n, buf, rec * count, ctypes.byref(ln)) == 0
    assert ln.value == rec * count
    raw = buf.raw
    for i in range(count):
        g, f = struct.unpack_from("<ii", raw, i * rec)
        pos = struct.unpack_from("<%dH" % n, raw, i * rec + 8)
        parenti = struct.unpack_from("<i", raw, i * rec + 8 + 2 * n)[0]
        assert (g, f, parenti) == (arr[i].g, arr[i].f, arr[i].parent_mask)
        assert list(pos) == list(arr[i].pos[:n])
    # through a frame and back
    rc, back = decode(encode(raw))
    assert rc == 0 and back[:-1] == raw
    out = (nat.pastar_node * count)()
    c = ctypes.c_int()
    assert L.pastar_wire_unpack_nodes(back, len(raw), n, out, count, ctypes.byref(c)) == 0 and c.value == count
    for i in range(count):
        assert (out[i].g, out[i].f, out[i].parent_mask, list(out[i].pos[:n])) == \
            (arr[i].g, arr[i].f, arr[i].parent_mask, list(arr[i].pos[:n]))
    # a ragged length is rejected
    assert L.pastar_wire_unpack_nodes(back, len(raw) - 1, n, out, count, ctypes.byref(c)) < 0
    assert L.pastar_wire_pack_nodes(arr, count, n, buf, rec * count - 1, ctypes.byref(ln)) < 0


def test_python_mirror_round_trip():
    from mpi_pastar_msa_amd import Node, lz4_dec, lz4_en, pack_nodes, unpack_nodes
    nodes = [Node((3, 4, 5, 6), 120, 300, 0b1011), Node((0, 0, 0, 1), 30, 280, 0b1000)]
    raw = pack_nodes(nodes, 4)
    assert len(raw) == 2 * (12 + 8)
    frame = lz4_en(raw)
    back = lz4_dec(frame)
    assert back == raw + b"\0"
    assert unpack_nodes(back[:-1], 4) == nodes
