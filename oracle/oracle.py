"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/liboracle.so (oracle/gcz_oracle.c, the plain-C
restatement of the reference's shared_tree build).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")


def build():
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


if not os.path.exists(LIB_PATH):
    build()
_lib = ctypes.CDLL(LIB_PATH)
_P, _U64, _U32, _I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
for name, res, args in [
    ("orc_nac", _I, [_I]),
    ("orc_leaf_transposed", _U64, [_U64]),
    ("orc_leaf_mirrored", _U64, [_U64, _I]),
    ("orc_leaf_canonical", _U64, [_U64, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    ("orc_ptr_xf", _U32, [_U32, _I, _I]),
    ("orc_node_canonical", None, [_U32, _U32, ctypes.POINTER(_U32), ctypes.POINTER(_U32),
                                  ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    ("orc_fasta_extract", _U64, [_P, _U64, _I, _U64, _P]),
    ("orc_pack", ctypes.c_int64, [_P, _U64, _I, _P]),
    ("orc_build", _P, [_P, _U64, _I]),
    ("orc_build_segmented", _P, [_P, _U64, _I, _U64]),
    ("orc_free", None, [_P]),
    ("orc_n_layers", _I, [_P]),
    ("orc_n_leaves", _U64, [_P]),
    ("orc_layer_size", _U64, [_P, _I]),
    ("orc_root", _U32, [_P]),
    ("orc_copy_leaves", None, [_P, _P]),
    ("orc_copy_layer", None, [_P, _I, _P]),
    ("orc_sort_tree", None, [_P]),
    ("orc_bytes", _U64, [_P]),
    ("orc_serialize", _U64, [_P, _P, _U64]),
    ("orc_width", _U64, [_P]),
]:
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = args
lib = _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


class OracleError(RuntimeError):
    def __init__(self, symbol, offset):
        super().__init__(f"Encountered unknown symbol: {symbol} (ASCII code {symbol})")
        self.symbol, self.offset = symbol, offset


class OracleTree:
    def __init__(self, h, L):
        self._h, self.L = h, L

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orc_free(self._h)
            self._h = None

    @property
    def n_layers(self):
        return _lib.orc_n_layers(self._h)

    @property
    def depth(self):
        return self.n_layers + 1

    @property
    def root(self):
        return _lib.orc_root(self._h)

    def leaves(self):
        n = _lib.orc_n_leaves(self._h)
        out = np.empty(n, dtype=np.uint64)
        _lib.orc_copy_leaves(self._h, _ptr(out))
        return out

    def layer(self, k):
        n = _lib.orc_layer_size(self._h, k)
        out = np.empty(2 * n, dtype=np.uint32)
        _lib.orc_copy_layer(self._h, k, _ptr(out))
        return out

    def layer_sizes(self):
        return [int(_lib.orc_layer_size(self._h, k)) for k in range(self.n_layers)]

    def sort(self):
        _lib.orc_sort_tree(self._h)

    def bytes(self):
        return int(_lib.orc_bytes(self._h))

    def width(self):
        return int(_lib.orc_width(self._h))

    def serialize(self):
        n = self.bytes()
        buf = np.empty(max(n, 1), dtype=np.uint8)
        assert _lib.orc_serialize(self._h, _ptr(buf), n) == n
        return buf[:n].tobytes()

    def leaves_bin(self):
        return self.leaves().astype("<u8").tobytes()

    def layers_bin(self):
        parts = []
        for k in range(self.n_layers):
            w = self.layer(k)
            parts.append(np.uint64(len(w) // 2).astype("<u8").tobytes())
            parts.append(w.astype("<u4").tobytes())
        return b"".join(parts)


def fasta_extract(data: bytes, L: int = 12, buffer_strands: int = 0) -> bytes:
    """fasta_reader's bases (buffer_strands 0 = the reference default 1 << 22)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    out = np.empty(max(len(data), 1), dtype=np.uint8)
    n = _lib.orc_fasta_extract(_ptr(buf), len(data), L, buffer_strands, _ptr(out))
    return out[:n].tobytes()


def pack(bases: bytes, L: int) -> np.ndarray:
    """Leaves of the truncated base string; raises OracleError like to_nac's exit(1)."""
    S = len(bases) // L
    buf = np.frombuffer(bases, dtype=np.uint8)
    out = np.empty(S, dtype=np.uint64)
    bad = _lib.orc_pack(_ptr(buf), S, L, _ptr(out))
    if bad >= 0:
        ch = bases[bad]
        sym = ord(chr(ch).upper()) if 97 <= ch <= 122 else ch
        raise OracleError(sym, bad)
    return out


def build_leaves(leaves: np.ndarray, L: int) -> OracleTree:
    a = np.ascontiguousarray(leaves, dtype=np.uint64)
    h = _lib.orc_build(_ptr(a), a.size, L)
    if not h:
        raise ValueError("empty input or bad L")
    return OracleTree(h, L)


def build_fasta(data: bytes, L: int) -> OracleTree:
    return build_leaves(pack(fasta_extract(data, L), L), L)


def build_leaves_segmented(leaves: np.ndarray, L: int, B: int) -> OracleTree:
    """tree_constructor::reduce over buffers of B strands (every buffer its own subtree)."""
    a = np.ascontiguousarray(leaves, dtype=np.uint64)
    h = _lib.orc_build_segmented(_ptr(a), a.size, L, B)
    if not h:
        raise ValueError("empty input or bad L / B")
    return OracleTree(h, L)


def reader_buffer_strands(nbytes: int, L: int, buffer_strands: int = 0) -> int:
    """fasta_reader's buffer size in strands (src/fasta_reader.cpp:21-31)."""
    return min(nbytes // L + 1, buffer_strands or (1 << 22))


def build_fasta_buffered(data: bytes, L: int, buffer_strands: int, first_strand: int = 0) -> OracleTree:
    """shared_tree{fasta_reader{path, buffer_strands}}: the reader's line contract and its
    buffers as subtrees (first_strand: buffers already read out)."""
    B = reader_buffer_strands(len(data), L, buffer_strands)
    leaves = pack(fasta_extract(data, L, buffer_strands), L)[first_strand:]
    return build_leaves_segmented(leaves, L, B)


def digest(tree) -> dict:
    """Hashes in the format of tests/golden/manifest.json (sorts the tree!)."""
    sha = lambda b: hashlib.sha256(b).hexdigest()
    d = {"n_leaves": len(tree.leaves()), "depth": tree.depth, "root": tree.root, "width": tree.width(),
         "layer_sizes": tree.layer_sizes(), "sha_leaves_bin": sha(tree.leaves_bin()),
         "sha_layers_bin": sha(tree.layers_bin()), "unsorted_bytes": tree.bytes(),
         "sha_unsorted_dag": sha(tree.serialize())}
    tree.sort()
    d["bytes"] = tree.bytes()
    d["sha_dag"] = sha(tree.serialize())
    return d
