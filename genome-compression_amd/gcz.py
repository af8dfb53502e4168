"""ctypes binding of libgcz (include/gcz.h) — the MI355X shared_tree build.

Python mirror of the reference's construction surface for tests and the bench:
`Context.build_fasta` corresponds to ``shared_tree{path}`` (compress.cpp:183),
`Context.build_leaves` to ``shared_tree(std::vector<dna>&)``
(src/shared_tree.cpp:212-215), and `Tree` to the container operations that
follow (sort_tree, bytes, serialize, width; src/shared_tree.cpp:316-513).

The library is the only compute path: if libgcz.so is missing this module
raises at import time (there is no CPU fallback).
"""
import ctypes
import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgcz.so")

GCZ_OK, GCZ_ERR_SYMBOL, GCZ_ERR_IO, GCZ_ERR_CAPACITY, GCZ_ERR_DEVICE, GCZ_ERR_ARG, GCZ_ERR_EMPTY = range(7)
NULL_WORD = 0x9FFFFFFF
MAX_LAYERS = 64


class GczError(RuntimeError):
    def __init__(self, code, msg, info=None):
        super().__init__(f"libgcz error {code}: {msg}")
        self.code = code
        self.info = info


class _Info(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int), ("L", ctypes.c_int), ("n_layers", ctypes.c_int),
                ("root", ctypes.c_uint32), ("n_strands", ctypes.c_uint64), ("n_leaves", ctypes.c_uint64),
                ("layer_size", ctypes.c_uint64 * MAX_LAYERS), ("error_offset", ctypes.c_uint64),
                ("error_symbol", ctypes.c_int), ("build_ms", ctypes.c_double), ("hashed_pairs", ctypes.c_uint64),
                ("bucketed_pairs", ctypes.c_uint64), ("leaf_path", ctypes.c_uint32), ("attempts", ctypes.c_uint32),
                ("build_ms_all", ctypes.c_double), ("repetitive", ctypes.c_uint32),
                ("handed_back", ctypes.c_uint32)]


if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built: run `make -C genome-compression_amd` "
                      "(or __graft_entry__.build()); there is no fallback path")
_lib = ctypes.CDLL(LIB_PATH)

_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_SIGS = {
    "gcz_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "gcz_ctx_destroy": (None, [_P]),
    "gcz_ctx_set_stream": (ctypes.c_int, [_P, _P]),
    "gcz_ctx_stream": (_P, [_P]),
    "gcz_ctx_last_error": (ctypes.c_char_p, [_P]),
    "gcz_dev_alloc": (_P, [_P, _U64]),
    "gcz_dev_free": (ctypes.c_int, [_P, _P]),
    "gcz_memcpy_h2d": (ctypes.c_int, [_P, _P, _P, _U64]),
    "gcz_upload_reserve": (ctypes.c_int, [_P, _U64]),
    "gcz_memcpy_d2h": (ctypes.c_int, [_P, _P, _P, _U64]),
    "gcz_ctx_sync": (ctypes.c_int, [_P]),
    "gcz_build_device_bases": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "gcz_build_device_leaves": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "gcz_build_host_fasta": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "gcz_build_host_fasta_buffered": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int, _U64, _U64]),
    "gcz_build_device_fasta_buffered": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int, _U64, _U64]),
    "gcz_build_host_leaves": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "gcz_build_device_fasta": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "gcz_fasta_extract_device": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int, _U64, _P, _U64, ctypes.POINTER(_U64)]),
    "gcz_info_get": (ctypes.c_int, [_P, ctypes.POINTER(_Info)]),
    "gcz_copy_leaves": (ctypes.c_int, [_P, _P]),
    "gcz_copy_layer": (ctypes.c_int, [_P, ctypes.c_int, _P]),
    "gcz_fetch_host": (ctypes.c_int, [_P, _P, _P]),
    "gcz_fetch_reserve": (ctypes.c_int, [_P, _U64]),
    "gcz_host_alloc": (_P, [_U64]),
    "gcz_host_free": (None, [_P, _U64]),
    "gcz_host_prefault": (ctypes.c_int, [_U64, ctypes.c_int]),
    "gcz_host_pool_release": (None, [ctypes.c_int]),
    "gcz_device_leaves": (_P, [_P]),
    "gcz_device_layer": (_P, [_P, ctypes.c_int]),
    "gcz_profile_enable": (ctypes.c_int, [_P, ctypes.c_int]),
    "gcz_profile_entry": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.POINTER(_U64), ctypes.POINTER(ctypes.c_double)]),
    "gcz_profile_reset": (None, [_P]),
    "gcz_profile_trace": (_U64, [_P, _P, _U64]),
    "gcz_tree_new": (_P, []),
    "gcz_tree_free": (None, [_P]),
    "gcz_tree_fetch": (ctypes.c_int, [_P, _P]),
    "gcz_tree_n_layers": (ctypes.c_int, [_P]),
    "gcz_tree_n_leaves": (_U64, [_P]),
    "gcz_tree_layer_size": (_U64, [_P, ctypes.c_int]),
    "gcz_tree_root": (ctypes.c_uint32, [_P]),
    "gcz_tree_L": (ctypes.c_int, [_P]),
    "gcz_tree_leaves": (_P, [_P]),
    "gcz_tree_layer": (_P, [_P, ctypes.c_int]),
    "gcz_tree_sort": (None, [_P]),
    "gcz_tree_bytes": (_U64, [_P]),
    "gcz_tree_serialize": (_U64, [_P, _P, _U64]),
    "gcz_tree_width": (_U64, [_P]),
    "gcz_tree_set_leaves": (None, [_P, ctypes.c_int, _P, _U64]),
    "gcz_tree_push_layer": (None, [_P, _P, _U64]),
    "gcz_tree_set_root": (None, [_P, ctypes.c_uint32]),
    "gcz_tree_deserialize": (ctypes.c_int, [_P, ctypes.c_int, _P, _U64]),
    "gcz_fasta_extract": (_U64, [_P, _U64, ctypes.c_int, _U64, _P]),
    "gcz_synth_fill": (None, [_P, ctypes.c_int, _U64, _U64, _U64]),
    "gcz_synth_default_seed": (_U64, []),
    "gcz_sort_device": (ctypes.c_int, [_P]),
    "gcz_sort_reserve": (ctypes.c_int, [_P]),
    "gcz_bytes_device": (ctypes.c_int, [_P, ctypes.POINTER(_U64)]),
    "gcz_serialize_device": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "gcz_device_dag": (_P, [_P, ctypes.POINTER(_U64)]),
    "gcz_decompress_device": (ctypes.c_int, [_P, _P, _U64]),
    "gcz_decompress": (ctypes.c_int, [_P, _P, _U64]),
    "gcz_dist_unique_id": (ctypes.c_int, [_P, _U64]),
    "gcz_group_create_rccl": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _P, ctypes.POINTER(_P)]),
    "gcz_group_create_shm": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _U64,
                                            ctypes.POINTER(_P)]),
    "gcz_group_create_local": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]),
    "gcz_group_destroy": (None, [_P]),
    "gcz_group_world": (ctypes.c_int, [_P]),
    "gcz_group_has_bulk": (ctypes.c_int, [_P]),
    "gcz_ctx_canary_check": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_uint64]),
    "gcz_group_canary_check": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_uint64]),
    "gcz_ctx_canary_selftest": (ctypes.c_int, [_P]),
    "gcz_group_n_local": (ctypes.c_int, [_P]),
    "gcz_group_rank": (ctypes.c_int, [_P, ctypes.c_int]),
    "gcz_group_ctx": (_P, [_P, ctypes.c_int]),
    "gcz_group_last_error": (ctypes.c_char_p, [_P]),
    "gcz_group_assemble": (ctypes.c_int, [_P, _P]),
    "gcz_group_xlog": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_U64), ctypes.POINTER(ctypes.c_char_p),
                                      ctypes.c_int]),
    "gcz_dist_p2p_plan": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U64), ctypes.c_int, _U64,
                                         ctypes.POINTER(_U64), ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "gcz_dist_gather_plan": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U64), _U64,
                                            ctypes.POINTER(_U64)]),
    "gcz_dist_watch_selftest": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "gcz_dist_plan": (ctypes.c_int, [_U64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U64), ctypes.POINTER(_U64),
                                      ctypes.POINTER(ctypes.c_int)]),
    "gcz_group_build_device_bases": (ctypes.c_int, [_P, ctypes.POINTER(_P), _U64, ctypes.c_int]),
    "gcz_group_build_device_leaves": (ctypes.c_int, [_P, ctypes.POINTER(_P), _U64, ctypes.c_int]),
    "gcz_group_info": (ctypes.c_int, [_P, ctypes.POINTER(_Info)]),
    "gcz_group_slice": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "gcz_group_copy_slice": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, _P]),
    "gcz_group_fetch": (ctypes.c_int, [_P, _P]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


# ---- host utilities ---------------------------------------------------------
def fasta_extract(data: bytes, L: int = 12, buffer_strands: int = 0) -> bytes:
    """Concatenated bases under the reference reader's line contract, for leaves of
    L nucleotides read through buffers of buffer_strands strands (0 = 1 << 22)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    out = np.empty(max(len(data), 1), dtype=np.uint8)
    n = _lib.gcz_fasta_extract(_ptr(buf), len(data), L, buffer_strands, _ptr(out))
    return out[:n].tobytes()


def synth(kind: int, nbases: int, seed: int = None) -> np.ndarray:
    """Synthetic genome (csrc/synth.h): kind 0 uniform ACGT, kind 1 tandem repeats."""
    if seed is None:
        seed = _lib.gcz_synth_default_seed()
    out = np.empty(max(nbases, 1), dtype=np.uint8)
    _lib.gcz_synth_fill(_ptr(out), kind, seed, 0, nbases)
    return out[:nbases]


# ---- host tree ----------------------------------------------------------------
class Tree:
    """Host-resident shared tree (leaves, per-layer node words, root)."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.gcz_tree_free(self._h)
            self._h = None

    @property
    def L(self):
        return _lib.gcz_tree_L(self._h)

    @property
    def n_layers(self):
        return _lib.gcz_tree_n_layers(self._h)

    @property
    def depth(self):
        return self.n_layers + 1

    @property
    def root(self):
        return _lib.gcz_tree_root(self._h)

    @classmethod
    def from_arrays(cls, L, leaves, layers, root):
        """Host tree from raw arrays (no GPU involved)."""
        t = cls(_lib.gcz_tree_new())
        lv = np.ascontiguousarray(leaves, dtype=np.uint64)
        _lib.gcz_tree_set_leaves(t._h, L, _ptr(lv), lv.size)
        for w in layers:
            w = np.ascontiguousarray(w, dtype=np.uint32)
            _lib.gcz_tree_push_layer(t._h, _ptr(w), w.size // 2)
        _lib.gcz_tree_set_root(t._h, int(root))
        return t

    @classmethod
    def deserialize(cls, data: bytes, L=12):
        t = cls(_lib.gcz_tree_new())
        buf = np.frombuffer(data, dtype=np.uint8)
        rc = _lib.gcz_tree_deserialize(t._h, L, _ptr(buf), len(data))
        if rc != GCZ_OK:
            raise GczError(rc, "malformed .dag")
        return t

    def leaves(self) -> np.ndarray:
        n = _lib.gcz_tree_n_leaves(self._h)
        if n == 0:
            return np.zeros(0, dtype=np.uint64)
        p = _lib.gcz_tree_leaves(self._h)
        return np.ctypeslib.as_array((ctypes.c_uint64 * n).from_address(p)).copy()

    def layer(self, k) -> np.ndarray:
        n = 2 * _lib.gcz_tree_layer_size(self._h, k)
        if n == 0:
            return np.zeros(0, dtype=np.uint32)
        p = _lib.gcz_tree_layer(self._h, k)
        return np.ctypeslib.as_array((ctypes.c_uint32 * n).from_address(p)).copy()

    def layer_sizes(self):
        return [int(_lib.gcz_tree_layer_size(self._h, k)) for k in range(self.n_layers)]

    def sort(self):
        _lib.gcz_tree_sort(self._h)

    def bytes(self):
        return int(_lib.gcz_tree_bytes(self._h))

    def width(self):
        return int(_lib.gcz_tree_width(self._h))

    def serialize(self) -> bytes:
        n = self.bytes()
        buf = np.empty(max(n, 1), dtype=np.uint8)
        got = _lib.gcz_tree_serialize(self._h, _ptr(buf), n)
        assert got == n
        return buf[:n].tobytes()

    # dump format of oracle/ref_harness.cpp
    def leaves_bin(self) -> bytes:
        return self.leaves().astype("<u8").tobytes()

    def layers_bin(self) -> bytes:
        out = []
        for k in range(self.n_layers):
            w = self.layer(k)
            out.append(np.uint64(len(w) // 2).astype("<u8").tobytes())
            out.append(w.astype("<u4").tobytes())
        return b"".join(out)


def dist_plan(S: int, world: int, rank: int):
    """Strands [s0, s1) owned by `rank` and the number G of distributed node levels."""
    s0, s1, g = _U64(), _U64(), ctypes.c_int()
    rc = _lib.gcz_dist_plan(S, world, rank, ctypes.byref(s0), ctypes.byref(s1), ctypes.byref(g))
    if rc != GCZ_OK:
        raise GczError(rc, "gcz_dist_plan: bad arguments")
    return int(s0.value), int(s1.value), int(g.value)


def _u64s(a):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    return a, a.ctypes.data_as(ctypes.POINTER(_U64))


def p2p_plan(world: int, me: int, M, reverse: bool, elem: int, sd=None, rd=None) -> np.ndarray:
    """The RCCL transport's transfers for rank `me` of an all-to-all (gcz_dist_p2p_plan):
    rows q = {send offset, send bytes, receive offset, receive bytes, q} in bytes."""
    Ma, Mp = _u64s(np.asarray(M).reshape(-1))
    keep = [Ma]
    sdp = rdp = None
    if sd is not None:
        a, sdp = _u64s(np.asarray(sd).reshape(-1))
        keep.append(a)
    if rd is not None:
        a, rdp = _u64s(np.asarray(rd).reshape(-1))
        keep.append(a)
    out = np.zeros(5 * world, dtype=np.uint64)
    rc = _lib.gcz_dist_p2p_plan(world, me, Mp, int(bool(reverse)), elem, sdp, rdp,
                                out.ctypes.data_as(ctypes.POINTER(_U64)))
    if rc != GCZ_OK:
        raise GczError(rc, "gcz_dist_p2p_plan: bad arguments")
    return out.reshape(world, 5)


def gather_plan(world: int, me: int, cnt, elem: int) -> np.ndarray:
    """The RCCL transport's transfers for rank `me` of the gather to rank 0 (same rows)."""
    c, cp = _u64s(cnt)
    out = np.zeros(5 * world, dtype=np.uint64)
    rc = _lib.gcz_dist_gather_plan(world, me, cp, elem, out.ctypes.data_as(ctypes.POINTER(_U64)))
    if rc != GCZ_OK:
        raise GczError(rc, "gcz_dist_gather_plan: bad arguments")
    return out.reshape(world, 5)


def dist_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    rc = _lib.gcz_dist_unique_id(buf, 128)
    if rc != GCZ_OK:
        raise GczError(rc, "gcz_dist_unique_id failed (RCCL not loadable)")
    return buf.raw


def _info_dict(i):
    return {"status": i.status, "L": i.L, "n_layers": i.n_layers, "root": i.root,
            "n_strands": i.n_strands, "n_leaves": i.n_leaves,
            "layer_size": [int(i.layer_size[k]) for k in range(i.n_layers)],
            "error_offset": i.error_offset, "error_symbol": i.error_symbol, "build_ms": i.build_ms,
            "hashed_pairs": i.hashed_pairs, "bucketed_pairs": i.bucketed_pairs, "leaf_path": i.leaf_path, "repetitive": i.repetitive, "handed_back": i.handed_back,
            "attempts": i.attempts, "build_ms_all": i.build_ms_all}


def _sha(b):
    return hashlib.sha256(b).hexdigest()


def digest(tree: Tree) -> dict:
    """Hashes in the format of tests/golden/manifest.json (sorts the tree!)."""
    d = {"n_leaves": int(_lib.gcz_tree_n_leaves(tree._h)), "depth": tree.depth, "root": tree.root,
         "width": tree.width(), "layer_sizes": tree.layer_sizes(),
         "sha_leaves_bin": _sha(tree.leaves_bin()), "sha_layers_bin": _sha(tree.layers_bin()),
         "unsorted_bytes": tree.bytes(), "sha_unsorted_dag": _sha(tree.serialize())}
    tree.sort()
    d["bytes"] = tree.bytes()
    d["sha_dag"] = _sha(tree.serialize())
    return d


# ---- device context -----------------------------------------------------------
def _canary(fn, h) -> str:
    msg = ctypes.create_string_buffer(2048)
    n = fn(h, msg, len(msg))
    if n < 0:
        raise GczError(n, "canary check: the context was created without GCZ_CANARY=1")
    return msg.value.decode() if n else ""


class DeviceBuffer:
    """Device allocation made through libgcz (no other GPU runtime needed)."""

    def __init__(self, ctx, nbytes):
        self._ctx = ctx
        self.nbytes = nbytes
        self.ptr = _lib.gcz_dev_alloc(ctx._h, nbytes)
        if not self.ptr:
            raise GczError(GCZ_ERR_DEVICE, f"gcz_dev_alloc({nbytes}) failed")

    def free(self):
        if getattr(self, "ptr", None) and getattr(self._ctx, "_h", None):
            _lib.gcz_dev_free(self._ctx._h, ctypes.c_void_p(self.ptr))
        self.ptr = None

    __del__ = free



class Context:
    """One GPU, one stream, a reusable workspace (gcz_ctx)."""

    def __init__(self, device: int = 0, _borrowed=None):
        self._owned = _borrowed is None
        if _borrowed is not None:
            self._h = ctypes.c_void_p(_borrowed)
            return
        h = ctypes.c_void_p()
        rc = _lib.gcz_ctx_create(device, ctypes.byref(h))
        if rc != GCZ_OK:
            raise GczError(rc, f"gcz_ctx_create(device={device}) failed")
        self._h = h

    def canary_check(self) -> str:
        """'' when every guard band of this context's buffers is intact (GCZ_CANARY=1 at
        creation), else a description of the overwritten ones."""
        return _canary(_lib.gcz_ctx_canary_check, self._h)

    def close(self):
        if getattr(self, "_h", None) and getattr(self, "_owned", True):
            _lib.gcz_ctx_destroy(self._h)
        self._h = None

    __del__ = close

    def _check(self, rc):
        if rc != GCZ_OK:
            raise GczError(rc, _lib.gcz_ctx_last_error(self._h).decode(), self.info())
        return self.info()

    def set_stream(self, stream_ptr: int):
        _lib.gcz_ctx_set_stream(self._h, ctypes.c_void_p(stream_ptr))

    @property
    def stream(self):
        return _lib.gcz_ctx_stream(self._h)

    def upload(self, host: np.ndarray) -> "DeviceBuffer":
        """Copy a host array into a new device buffer owned by this context."""
        a = np.ascontiguousarray(host)
        buf = DeviceBuffer(self, a.nbytes)
        rc = _lib.gcz_memcpy_h2d(self._h, ctypes.c_void_p(buf.ptr), _ptr(a), a.nbytes)
        if rc != GCZ_OK:
            raise GczError(rc, "H2D copy failed")
        return buf

    def sync(self):
        rc = _lib.gcz_ctx_sync(self._h)
        if rc != GCZ_OK:
            raise GczError(rc, "stream synchronize failed")

    def info(self) -> dict:
        i = _Info()
        _lib.gcz_info_get(self._h, ctypes.byref(i))
        return _info_dict(i)

    def build_fasta(self, data: bytes, L: int = 12) -> dict:
        buf = np.frombuffer(data, dtype=np.uint8)
        return self._check(_lib.gcz_build_host_fasta(self._h, _ptr(buf), len(data), L))

    def build_fasta_buffered(self, data: bytes, L: int = 12, buffer_strands: int = 0, first_strand: int = 0) -> dict:
        """shared_tree{fasta_reader{path, buffer_strands}}: every reader buffer its own subtree."""
        buf = np.frombuffer(data, dtype=np.uint8)
        return self._check(_lib.gcz_build_host_fasta_buffered(self._h, _ptr(buf), len(data), L, buffer_strands,
                                                              first_strand))

    def build_device_fasta_buffered(self, dev_ptr: int, nbytes: int, L: int = 12, buffer_strands: int = 0,
                                    first_strand: int = 0) -> dict:
        return self._check(_lib.gcz_build_device_fasta_buffered(self._h, ctypes.c_void_p(dev_ptr), nbytes, L,
                                                                buffer_strands, first_strand))

    def build_leaves(self, leaves: np.ndarray, L: int = 12) -> dict:
        a = np.ascontiguousarray(leaves, dtype=np.uint64)
        return self._check(_lib.gcz_build_host_leaves(self._h, _ptr(a), a.size, L))

    def build_device_bases(self, dev_ptr: int, nbases: int, L: int = 12) -> dict:
        return self._check(_lib.gcz_build_device_bases(self._h, ctypes.c_void_p(dev_ptr), nbases, L))

    def build_device_fasta(self, dev_ptr: int, nbytes: int, L: int = 12) -> dict:
        """FASTA file bytes already in device memory: line contract + build on the device."""
        return self._check(_lib.gcz_build_device_fasta(self._h, ctypes.c_void_p(dev_ptr), nbytes, L))

    def fasta_extract_device(self, data: bytes, L: int = 12, buffer_strands: int = 0) -> bytes:
        """The device line contract on `data` (uploaded), bases back to the host."""
        buf = self.upload(np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8))
        try:
            n = _U64()
            out = DeviceBuffer(self, max(len(data), 1))
            rc = _lib.gcz_fasta_extract_device(self._h, ctypes.c_void_p(buf.ptr), len(data), L, buffer_strands,
                                               ctypes.c_void_p(out.ptr), max(len(data), 1), ctypes.byref(n))
            if rc != GCZ_OK:
                raise GczError(rc, "gcz_fasta_extract_device failed")
            host = np.empty(max(int(n.value), 1), dtype=np.uint8)
            if n.value:
                _lib.gcz_memcpy_d2h(self._h, _ptr(host), ctypes.c_void_p(out.ptr), int(n.value))
            out.free()
            return host[:int(n.value)].tobytes()
        finally:
            buf.free()

    def build_device_leaves(self, dev_ptr: int, S: int, L: int = 12) -> dict:
        return self._check(_lib.gcz_build_device_leaves(self._h, ctypes.c_void_p(dev_ptr), S, L))

    def tree(self) -> Tree:
        t = _lib.gcz_tree_new()
        rc = _lib.gcz_tree_fetch(self._h, t)
        if rc != GCZ_OK:
            _lib.gcz_tree_free(t)
            raise GczError(rc, "gcz_tree_fetch failed")
        return Tree(t)

    # ---- ratio path on the device (frequency sort, bytes(), .dag) ----
    def sort_device(self):
        """shared_tree::sort_tree on the device, in place on the last build."""
        rc = _lib.gcz_sort_device(self._h)
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_sort_device: " + _lib.gcz_ctx_last_error(self._h).decode())

    def bytes_device(self) -> int:
        out = _U64()
        rc = _lib.gcz_bytes_device(self._h, ctypes.byref(out))
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_bytes_device failed")
        return int(out.value)

    def serialize_device(self) -> bytes:
        """The .dag bytes written on the device (shared_tree::serialize)."""
        n = _U64()
        _lib.gcz_serialize_device(self._h, None, 0, ctypes.byref(n))
        buf = np.empty(max(int(n.value), 1), dtype=np.uint8)
        rc = _lib.gcz_serialize_device(self._h, _ptr(buf), buf.size, ctypes.byref(n))
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_serialize_device failed")
        return buf[:int(n.value)].tobytes()

    def decompress(self) -> bytes:
        """The genome the last build represents (upper-case IUPAC, S*L symbols), decoded on the device."""
        i = self.info()
        n = i["n_strands"] * i["L"]
        buf = np.empty(max(n, 1), dtype=np.uint8)
        rc = _lib.gcz_decompress(self._h, _ptr(buf), n)
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_decompress failed")
        return buf[:n].tobytes()

    def profile(self, on=True):
        _lib.gcz_profile_enable(self._h, int(on))

    def profile_reset(self):
        _lib.gcz_profile_reset(self._h)

    def profile_table(self) -> dict:
        out = {}
        k = 0
        name = ctypes.c_char_p()
        n = ctypes.c_uint64()
        ms = ctypes.c_double()
        while _lib.gcz_profile_entry(self._h, k, ctypes.byref(name), ctypes.byref(n), ctypes.byref(ms)) == 0:
            out[name.value.decode()] = {"launches": int(n.value), "total_ms": float(ms.value)}
            k += 1
        return out

    def profile_trace(self) -> list:
        """Profiled scopes since the last reset, in stream order: (name, start ms after the
        build's start event, duration ms)."""
        names = list(self.profile_table())
        n = int(_lib.gcz_profile_trace(self._h, None, 0))
        buf = np.empty(max(3 * n, 3), dtype=np.float32)
        n = min(n, int(_lib.gcz_profile_trace(self._h, _ptr(buf), n)))
        return [(names[int(buf[3 * i])], float(buf[3 * i + 1]), float(buf[3 * i + 2])) for i in range(n)]


# ---- multi-rank build -----------------------------------------------------------
class Group:
    """Ranks of a multi-rank build (gcz_group): `Group.local(world)` runs `world`
    virtual ranks on one device (tests); `Group.rccl(ctx, rank, world, uid)` is one
    rank per process and GPU (bench).  Rank r owns strands dist_plan(S, world, r)."""

    def __init__(self, handle, keep=None):
        self._h = handle
        self._keep = keep

    @classmethod
    def local(cls, world: int, device: int = 0):
        h = ctypes.c_void_p()
        rc = _lib.gcz_group_create_local(device, world, ctypes.byref(h))
        if rc != GCZ_OK:
            raise GczError(rc, f"gcz_group_create_local(world={world}) failed")
        return cls(h)

    @classmethod
    def rccl(cls, ctx: Context, rank: int, world: int, unique_id: bytes):
        h = ctypes.c_void_p()
        uid = ctypes.create_string_buffer(unique_id, 128)
        rc = _lib.gcz_group_create_rccl(ctx._h, rank, world, uid, ctypes.byref(h))
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_group_create_rccl failed: " + _lib.gcz_ctx_last_error(ctx._h).decode())
        return cls(h, keep=ctx)

    @classmethod
    def shm(cls, ctx: Context, rank: int, world: int, name: str, region_bytes: int = 1 << 30):
        """One rank per process on a shared device, exchanges host-staged through the
        POSIX shared-memory object `name` (testing the multi-process path on one GPU)."""
        h = ctypes.c_void_p()
        rc = _lib.gcz_group_create_shm(ctx._h, rank, world, name.encode(), region_bytes, ctypes.byref(h))
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_group_create_shm failed: " + _lib.gcz_ctx_last_error(ctx._h).decode())
        return cls(h, keep=ctx)

    def close(self):
        if getattr(self, "_h", None):
            _lib.gcz_group_destroy(self._h)
            self._h = None

    __del__ = close

    @property
    def world(self):
        return _lib.gcz_group_world(self._h)

    @property
    def n_local(self):
        return _lib.gcz_group_n_local(self._h)

    @property
    def has_bulk(self) -> bool:
        """Bulk groups run on a second stream (gcz_group_has_bulk)."""
        return bool(_lib.gcz_group_has_bulk(self._h))

    def canary_check(self) -> str:
        """'' when every guard band of every local rank's buffers is intact (GCZ_CANARY=1 at
        creation), else a description of the overwritten ones."""
        return _canary(_lib.gcz_group_canary_check, self._h)

    def rank(self, i=0):
        return _lib.gcz_group_rank(self._h, i)

    def ctx(self, i=0) -> Context:
        return Context(_borrowed=_lib.gcz_group_ctx(self._h, i))

    def build_device_bases(self, dev_ptrs, S: int, L: int = 12) -> dict:
        arr = (ctypes.c_void_p * len(dev_ptrs))(*[ctypes.c_void_p(p) for p in dev_ptrs])
        rc = _lib.gcz_group_build_device_bases(self._h, arr, S, L)
        if rc != GCZ_OK:
            raise GczError(rc, _lib.gcz_group_last_error(self._h).decode(), self.info())
        return self.info()

    def build_device_leaves(self, dev_ptrs, S: int, L: int = 12) -> dict:
        arr = (ctypes.c_void_p * len(dev_ptrs))(*[ctypes.c_void_p(p) for p in dev_ptrs])
        rc = _lib.gcz_group_build_device_leaves(self._h, arr, S, L)
        if rc != GCZ_OK:
            raise GczError(rc, _lib.gcz_group_last_error(self._h).decode(), self.info())
        return self.info()

    def info(self) -> dict:
        i = _Info()
        _lib.gcz_group_info(self._h, ctypes.byref(i))
        return _info_dict(i)

    def slice(self, i: int, layer: int):
        off, cnt = _U64(), _U64()
        rc = _lib.gcz_group_slice(self._h, i, layer, ctypes.byref(off), ctypes.byref(cnt))
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_group_slice failed")
        return int(off.value), int(cnt.value)

    def copy_slice(self, i: int, layer: int) -> np.ndarray:
        _, cnt = self.slice(i, layer)
        out = np.empty(cnt if layer < 0 else 2 * cnt, dtype=np.uint64 if layer < 0 else np.uint32)
        rc = _lib.gcz_group_copy_slice(self._h, i, layer, _ptr(out))
        if rc != GCZ_OK:
            raise GczError(rc, "gcz_group_copy_slice failed")
        return out

    def assemble(self, dst: "Context" = None) -> dict:
        """The last build's whole tree into `dst` (rank 0: a Context on its device other than
        the group's; other ranks pass None) in the single-device layout, so dst's device sort,
        .dag writer, decompression and tree() work on it (gcz_group_assemble)."""
        rc = _lib.gcz_group_assemble(self._h, dst._h if dst is not None else None)
        if rc != GCZ_OK:
            raise GczError(rc, _lib.gcz_group_last_error(self._h).decode())
        return dst.info() if dst is not None else {}

    def exchange_log(self, i=0) -> list:
        """The last build's exchanges as local rank i saw them (gcz_group_xlog): name, sequence
        number, bytes sent to / received from the other ranks, host enqueue time (us)."""
        n = _lib.gcz_group_xlog(self._h, i, None, None, 0)
        if n <= 0:
            return []
        rec = (_U64 * (4 * n))()
        names = (ctypes.c_char_p * n)()
        _lib.gcz_group_xlog(self._h, i, rec, names, n)
        return [{"seq": int(rec[4 * k]), "name": names[k].decode(), "sent": int(rec[4 * k + 1]),
                 "recvd": int(rec[4 * k + 2]), "t_us": int(rec[4 * k + 3])} for k in range(n)]

    def tree(self) -> Tree:
        t = _lib.gcz_tree_new()
        rc = _lib.gcz_group_fetch(self._h, t)
        if rc != GCZ_OK:
            _lib.gcz_tree_free(t)
            raise GczError(rc, "gcz_group_fetch failed")
        return Tree(t)
