"""Loader for tests/golden/ (MPICH 3.3.2 MPI_Pack outputs; see tools/make_golden.py)."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "mpich_golden.json")

_doc = None


def cases():
    global _doc
    if _doc is None:
        with open(GOLDEN) as f:
            _doc = json.load(f)
    return _doc["cases"]


def case(name):
    for c in cases():
        if c["name"] == name:
            return c
    raise KeyError(name)


def source_buffer(c):
    """The generator's input: byte i of the allocation = i & 0xFF."""
    return (np.arange(c["buflen"], dtype=np.int64) & 0xFF).astype(np.uint8)


def check_packed(c, packed):
    """Assert `packed` (bytes-like / uint8 array) equals the library's MPI_Pack."""
    b = bytes(np.asarray(packed, dtype=np.uint8).tobytes())
    assert len(b) == c["position"], f"{c['name']}: position {len(b)} != {c['position']}"
    if "packed_hex" in c:
        exp = bytes.fromhex(c["packed_hex"])
        if b != exp:
            i = next(k for k in range(len(b)) if b[k] != exp[k])
            raise AssertionError(f"{c['name']}: first mismatch at byte {i}: got {b[i]} expected {exp[i]}")
    else:
        assert b[:64].hex() == c["packed_head_hex"], f"{c['name']}: head mismatch"
        assert b[-64:].hex() == c["packed_tail_hex"], f"{c['name']}: tail mismatch"
        assert hashlib.sha256(b).hexdigest() == c["packed_sha256"], f"{c['name']}: sha256 mismatch"


def check_unpacked(c, buf):
    b = bytes(np.asarray(buf, dtype=np.uint8).tobytes())
    assert hashlib.sha256(b).hexdigest() == c["unpacked_sha256"], f"{c['name']}: unpack sha256 mismatch"
