"""ctypes binding of libbfhip.so (the C ABI in include/bfhip.h).

This is the only way the package reaches the engine: there is no CPU
fallback.  If the shared library is missing or fails to load, importing the
driver raises ``BfHipUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading
from typing import List, Optional, Tuple

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(PKG_DIR, "lib", "libbfhip.so")

BF_OK, BF_EINVAL, BF_ENOMEM, BF_EDEVICE, BF_ERCCL, BF_ERANGE = 0, 1, 2, 3, 4, 5
BF_IMPORT_REPLACE, BF_IMPORT_OR = 0, 1
BF_FLAG_ROUTE32 = 1
BF_FLAG_ENGINE_MD5, BF_FLAG_ENGINE_SHA1 = 2, 4   # RubyTest hash engines (ruby_test.rb:43-61)
BF_FLAG_ENCODER = 8   # no bitset: region-set encodes only (a replicated filter's second, encoding handle)
BF_MAX_K = 64
PROFILE_NAME_LEN = 64   # BF_PROFILE_NAME_LEN
DIRTY_BLOCK_BYTES = 65536   # BF_DIRTY_BLOCK_BYTES

_STATUS = {BF_EINVAL: "BF_EINVAL", BF_ENOMEM: "BF_ENOMEM", BF_EDEVICE: "BF_EDEVICE",
           BF_ERCCL: "BF_ERCCL", BF_ERANGE: "BF_ERANGE"}


class BfHipUnavailable(ImportError):
    """libbfhip.so could not be loaded (not built, or no HIP runtime)."""


class BfHipError(RuntimeError):
    """A non-argument failure reported by the engine (device, memory, collective)."""

    def __init__(self, code: int, msg: str):
        super().__init__("%s: %s" % (_STATUS.get(code, "BF_E%d" % code), msg))
        self.code = code


class ArgumentError(ValueError):
    """Mirror of Ruby's ArgumentError (raised where the reference raises it)."""


BF_MAX_DEVICES = 16
BF_MODE_REPLICATED, BF_MODE_PARTITIONED = 0, 1


class bf_config(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("batch_keys", ctypes.c_uint64), ("batch_bytes", ctypes.c_uint64),
                ("shard_count", ctypes.c_uint32), ("shard_index", ctypes.c_uint32),
                ("shard_block_log2", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("device_count", ctypes.c_uint32), ("mode", ctypes.c_uint32),
                ("devices", ctypes.c_int32 * BF_MAX_DEVICES)]


_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32

# name -> (restype, argtypes); must list every function declared in include/bfhip.h
SIGNATURES = {
    "bf_create": (ctypes.c_int, [_u64, _u32, ctypes.POINTER(bf_config), ctypes.POINTER(_vp)]),
    "bf_destroy": (ctypes.c_int, [_vp]),
    "bf_last_error": (ctypes.c_char_p, [_vp]),
    "bf_version": (ctypes.c_char_p, []),
    "bf_info": (ctypes.c_int, [_vp, _u64p, _u32p, _u64p, _u64p]),
    "bf_insert_many": (ctypes.c_int, [_vp, _vp, _vp, _u64, _u8p, _vp]),
    "bf_include_many": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "bf_indexes_many": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "bf_indexes": (ctypes.c_int, [_vp, _u64, _u64, _u32, _vp]),
    "bf_check_offsets": (ctypes.c_int, [_vp, _u64, _u64p]),
    "bf_clear": (ctypes.c_int, [_vp]),
    "bf_export_redis": (ctypes.c_int, [_vp, _vp, _u64, _u64p]),
    "bf_import_redis": (ctypes.c_int, [_vp, _vp, _u64, _u32]),
    "bf_insert_many_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "bf_include_many_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_indexes_many_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_device_bits": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), _u64p]),
    "bf_hash_many_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_insert_digests_dev": (ctypes.c_int, [_vp, _vp, _u64, _vp, _vp, _vp]),
    "bf_include_digests_dev": (ctypes.c_int, [_vp, _vp, _u64, _vp, _vp]),
    "bf_include_hash_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_region_sets_capacity": (ctypes.c_int, [_vp, _u64, _u64p]),
    "bf_encode_region_sets_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _u64, _vp]),
    "bf_encode_region_sets_digests_dev": (ctypes.c_int, [_vp, _vp, _u64, _vp, _u64, _vp]),
    "bf_insert_region_sets_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _u64, _vp, _vp, _vp]),
    "bf_insert_encode_region_sets_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _u64, _vp, _vp, _vp, _u64, _vp, _u64,
                                                        _vp]),
    "bf_insert_plan": (ctypes.c_int, [_vp, _u64, _u32p, _u64p]),
    "bf_track_dirty": (ctypes.c_int, [_vp, _u32]),
    "bf_dirty_ranges": (ctypes.c_int, [_vp, _u64p, _u32, _u32p, _u64p, _u32]),
    "bf_export_range": (ctypes.c_int, [_vp, _u64, _u64, _vp]),
    "bf_insert_many_changes": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _u64, _u64p]),
    "bf_profile": (ctypes.c_int, [_vp, _u32]),
    "bf_profile_read": (ctypes.c_int, [_vp, _vp, _vp, _vp, _u32, _u32p, _u32]),
    "bf_sync": (ctypes.c_int, [_vp]),
    "bf_stream": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "bf_shard_info": (ctypes.c_int, [_vp, _u32p, _u32p, _u32p, _u64p]),
    "bf_route_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp, _vp]),
    "bf_shard_insert_dev": (ctypes.c_int, [_vp, _vp, _u64, _vp, _vp]),
    "bf_shard_test_dev": (ctypes.c_int, [_vp, _vp, _u64, _vp, _vp]),
    "bf_combine_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_route_window_split": (ctypes.c_int, [_vp, _u32p]),
    "bf_route_windows_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    "bf_shard_insert_hi_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _vp]),
    "bf_shard_insert_windows_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _u32, _u32, _vp, _vp]),
    "bf_shard_test_windows_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _u32, _u32, _vp, _vp]),
    "bf_shard_test_hi_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _vp]),
    "bf_combine_windows_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _u32, _vp, _u64, _vp, _vp]),
    "bf_pack_segments_dev": (ctypes.c_int, [_vp, _vp, _vp, _u32, _u64, _vp, _vp]),
    "bf_combine_windows_packed_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _u32, _vp, _u64, _vp, _vp]),
    "bf_route_chunk_info": (ctypes.c_int, [_vp, _u64, _u64p, _u64p, _u32p]),
    "bf_route_chunks_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp, _u64, _u64, _vp]),
    "bf_shard_insert_chunks_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _u64, _u64, _vp, _u32, _vp, _vp]),
    "bf_shard_test_chunks_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _u64, _u64, _vp, _u32, _vp, _vp]),
    "bf_shard_test_chunks_packed_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _u64, _u64, _vp, _u32, _vp, _vp]),
    "bf_shard_insert_test_chunks_packed_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u32, _u64,
                                                              _u64, _u32, _vp, _vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_route_chunks_digests_dev": (ctypes.c_int, [_vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp, _u64, _u64, _vp]),
    "bf_shard_test_chunks_hash_dev": (ctypes.c_int, [_vp, _vp, _u64, _u32, _vp, _u64, _u64, _vp, _u32, _vp,
                                                     _vp, _vp, _u64, _vp, _vp]),
    "bf_combine_chunks_packed_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _u64, _u64, _vp, _u64, _vp, _vp]),
    "bf_shard_export": (ctypes.c_int, [_vp, _vp, _u64, _u64p]),
    "bf_shard_import": (ctypes.c_int, [_vp, _vp, _u64, _u32]),
    "bf_lua_create": (ctypes.c_int, [ctypes.c_double, ctypes.c_double, ctypes.POINTER(bf_config),
                                     ctypes.POINTER(_vp)]),
    "bf_lua_destroy": (ctypes.c_int, [_vp]),
    "bf_lua_last_error": (ctypes.c_char_p, [_vp]),
    "bf_lua_insert_many": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _u64p]),
    "bf_lua_insert_many_changes": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _u64p, _vp, _u64, _u64p]),
    "bf_lua_include_many": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp]),
    "bf_lua_insert_many_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _u64p, _vp]),
    "bf_lua_include_many_dev": (ctypes.c_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "bf_lua_profile": (ctypes.c_int, [_vp, _u32]),
    "bf_lua_profile_read": (ctypes.c_int, [_vp, _vp, _vp, _vp, _u32, _u32p, _u32]),
    "bf_lua_clear": (ctypes.c_int, [_vp]),
    "bf_lua_get_count": (ctypes.c_int, [_vp, _u64p]),
    "bf_lua_set_count": (ctypes.c_int, [_vp, _u64]),
    "bf_lua_layers": (ctypes.c_int, [_vp, _u32p]),
    "bf_lua_export_layer": (ctypes.c_int, [_vp, _u32, _vp, _u64, _u64p]),
    "bf_lua_import_layer": (ctypes.c_int, [_vp, _u32, _vp, _u64]),
    "bf_lua_layer_params": (ctypes.c_int, [ctypes.c_double, ctypes.c_double, _u32, _u64p, _u32p]),
    "bf_lua_index": (ctypes.c_int, [ctypes.c_double, _u64, _u32p]),
    "bf_optimal_m": (ctypes.c_int64, [ctypes.c_double, ctypes.c_double]),
    "bf_optimal_k": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
}

_lib = None
_lib_lock = threading.Lock()


def lib_path() -> str:
    return os.environ.get("BFHIP_LIB", DEFAULT_LIB)


def _share_torch_runtime() -> None:
    """Make libbfhip bind to the HIP runtime PyTorch-ROCm already uses.

    torch ships its own ``libamdhip64.so`` (SONAME ``libamdhip64.so.7``) and
    links it by the unversioned name.  If libbfhip is loaded first, the system
    runtime comes in under that SONAME and torch later maps a SECOND runtime,
    after which torch sees no GPU.  Loading torch first lets the dynamic
    loader satisfy libbfhip's ``libamdhip64.so.7`` with torch's copy: one
    runtime, shared streams and device pointers.  BFHIP_STANDALONE=1 skips this
    (e.g. a process that never imports torch).
    """
    if os.environ.get("BFHIP_STANDALONE") == "1" or "torch" in sys.modules:
        return
    import importlib.util
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def load() -> ctypes.CDLL:
    """Load libbfhip.so once; raise BfHipUnavailable if it cannot be loaded."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        _share_torch_runtime()
        path = lib_path()
        if not os.path.exists(path):
            raise BfHipUnavailable(
                "libbfhip.so not found at %s — build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (or `make -C redis-bloomfilter_amd/csrc`)" % path)
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:  # missing HIP runtime etc.
            raise BfHipUnavailable("cannot load %s: %s" % (path, e)) from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def version() -> str:
    return load().bf_version().decode()


BF_OPTIMAL_M_INVALID = -(1 << 63)


def optimal_m(n, error_rate) -> int:
    m = int(load().bf_optimal_m(float(n), float(error_rate)))
    if m == BF_OPTIMAL_M_INVALID:   # Infinity/NaN: Float#round raises FloatDomainError in Ruby
        raise FloatingPointError("FloatDomainError: optimal_m(%r, %r) is not finite" % (n, error_rate))
    return m


def optimal_k(n: int, m: int) -> int:
    return int(load().bf_optimal_k(int(n), int(m)))


def indexes(key: bytes, m: int, k: int) -> List[int]:
    """One key's k offsets (Ruby#indexes_for, ruby.rb:41-55) through bf_indexes: the device
    kernel on the current GPU, no filter needed."""
    buf = np.frombuffer(bytes(key), np.uint8) if len(key) else np.zeros(1, np.uint8)
    out = np.zeros(max(int(k), 1), np.uint64)
    _check(load().bf_indexes(_ptr(buf), len(key), int(m), int(k), _ptr(out)))
    return [int(x) for x in out[: int(k)]]


def check_offsets(offsets: np.ndarray) -> None:
    """The key-offset rule every hashing kernel applies (bf_check_offsets): offsets[0..n]
    non-decreasing, every key below 2 GiB.  Raises ArgumentError naming the first bad key.
    Host-only: callers of the *_dev entry points can check their offsets before the upload."""
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    if offs.size == 0:
        raise ArgumentError("offsets needs n + 1 entries")
    bad = ctypes.c_uint64()
    _check(load().bf_check_offsets(_ptr(offs), offs.size - 1, ctypes.byref(bad)))


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data


def _check(code: int, h=None) -> None:
    if code == BF_OK:
        return
    lib = load()
    msg = lib.bf_last_error(h).decode(errors="replace") if lib else ""
    if code in (BF_EINVAL, BF_ERANGE):
        raise ArgumentError("%s: %s" % (_STATUS.get(code), msg))
    raise BfHipError(code, msg)


class Filter:
    """One device-resident filter (a `bf_handle*`).

    Arrays are numpy: ``keys`` uint8, ``offsets`` uint64 with n+1 entries.
    The ``*_dev`` methods take raw device addresses (ints), e.g. from
    ``torch.Tensor.data_ptr()``, and a hipStream_t as an int (``stream=None``:
    the filter's own stream; ``0`` is HIP's null stream, e.g. torch's default).
    """

    def __init__(self, m_bits: int, k: int, device: int = -1, batch_keys: int = 0,
                 batch_bytes: int = 0, shard_count: int = 1, shard_index: int = 0,
                 shard_block_log2: int = 0, flags: int = 0, devices=None, mode: str = "replicated"):
        """devices: a list of HIP ordinals -> one multi-device handle over them (bf_config
        device_count / devices / mode; ``mode`` "replicated" or "partitioned")."""
        self._lib = load()
        cfg = bf_config(ctypes.sizeof(bf_config), int(device), int(batch_keys), int(batch_bytes),
                        int(shard_count), int(shard_index), int(shard_block_log2), int(flags))
        if devices is not None:
            devices = [int(d) for d in devices]
            if not 0 < len(devices) <= BF_MAX_DEVICES:
                raise ArgumentError("devices must list 1..%d ordinals" % BF_MAX_DEVICES)
            if mode not in ("replicated", "partitioned"):
                raise ArgumentError("mode must be 'replicated' or 'partitioned'")
            cfg.device_count = len(devices)
            cfg.mode = BF_MODE_PARTITIONED if mode == "partitioned" else BF_MODE_REPLICATED
            for i, d in enumerate(devices):
                cfg.devices[i] = d
        self.devices = devices
        self.mode = mode if devices is not None else None
        self.route32 = bool(flags & BF_FLAG_ROUTE32)
        h = _vp()
        rc = self._lib.bf_create(int(m_bits), int(k), ctypes.byref(cfg), ctypes.byref(h))
        _check(rc, None)
        self._h = h
        m = ctypes.c_uint64()
        kk = ctypes.c_uint32()
        reach = ctypes.c_uint64()
        devb = ctypes.c_uint64()
        _check(self._lib.bf_info(h, ctypes.byref(m), ctypes.byref(kk), ctypes.byref(reach),
                                 ctypes.byref(devb)), h)
        self.m, self.k, self.reach_bits, self.device_bytes = m.value, kk.value, reach.value, devb.value
        self.device = int(device)
        sc, si, bl = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        lb = ctypes.c_uint64()
        _check(self._lib.bf_shard_info(h, ctypes.byref(sc), ctypes.byref(si), ctypes.byref(bl),
                                       ctypes.byref(lb)), h)
        self.shard_count, self.shard_index, self.block_log2, self.local_bits = sc.value, si.value, bl.value, lb.value

    # -- lifecycle
    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.bf_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        if not self._h:
            raise ArgumentError("filter is closed")
        return self._h

    # -- host-pointer batch API
    @staticmethod
    def _keys(keys: np.ndarray, offsets: np.ndarray) -> Tuple[np.ndarray, np.ndarray, int]:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        if offsets.ndim != 1 or len(offsets) < 1:
            raise ArgumentError("offsets must be a 1-D array of n+1 entries")
        n = len(offsets) - 1
        if n and int(offsets[-1]) > len(keys):
            raise ArgumentError("offsets point past the key buffer")
        if len(keys) == 0:
            keys = np.zeros(1, np.uint8)
        return keys, offsets, n

    def insert_many(self, keys: np.ndarray, offsets: np.ndarray, any_new: bool = False,
                    per_key_new: bool = False):
        keys, offsets, n = self._keys(keys, offsets)
        flag = ctypes.c_uint8(0)
        pk = np.zeros(max(n, 1), np.uint8) if per_key_new else None
        _check(self._lib.bf_insert_many(self.handle, _ptr(keys), _ptr(offsets), n,
                                        ctypes.byref(flag) if any_new else None, _ptr(pk)), self._h)
        return (bool(flag.value) if any_new else None), (pk[:n] if per_key_new else None)

    # bf_insert_many_changes limits (include/bfhip.h)
    CHANGES_MAX_PROBES = 4096
    CHANGES_MAX_BYTES = 64 << 10

    def insert_many_changes(self, keys: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        """Insert a small batch; returns the bit offsets it flipped 0 -> 1 (each once, uint64):
        the SETBITs that bring a Redis copy up to date (ruby.rb:57-63)."""
        keys, offsets, n = self._keys(keys, offsets)
        out = np.zeros(max(n * self.k, 1), np.uint64)
        cnt = ctypes.c_uint64(0)
        _check(self._lib.bf_insert_many_changes(self.handle, _ptr(keys), _ptr(offsets), n, _ptr(out), len(out),
                                                ctypes.byref(cnt)), self._h)
        return out[: cnt.value]

    def include_many(self, keys: np.ndarray, offsets: np.ndarray, out: Optional[np.ndarray] = None) -> np.ndarray:
        """include? of every key -> uint8 answers (1/0).  out: an optional caller-owned uint8
        buffer of >= n entries (reused across calls, its pages are already mapped)."""
        keys, offsets, n = self._keys(keys, offsets)
        if out is None:
            out = np.empty(max(n, 1), np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.ndim != 1 or len(out) < max(n, 1):
            raise ArgumentError("out must be a contiguous 1-D uint8 array of at least n entries")
        _check(self._lib.bf_include_many(self.handle, _ptr(keys), _ptr(offsets), n, _ptr(out)), self._h)
        return out[:n]

    def indexes_many(self, keys: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        keys, offsets, n = self._keys(keys, offsets)
        out = np.zeros(max(n * self.k, 1), np.uint64)
        _check(self._lib.bf_indexes_many(self.handle, _ptr(keys), _ptr(offsets), n, _ptr(out)), self._h)
        return out[: n * self.k].reshape(n, self.k)

    def clear(self) -> None:
        _check(self._lib.bf_clear(self.handle), self._h)

    def sync(self) -> None:
        _check(self._lib.bf_sync(self.handle), self._h)

    # -- Redis string
    def export_redis(self) -> bytes:
        n = ctypes.c_uint64(0)
        _check(self._lib.bf_export_redis(self.handle, None, 0, ctypes.byref(n)), self._h)
        buf = np.zeros(max(n.value, 1), np.uint8)
        _check(self._lib.bf_export_redis(self.handle, _ptr(buf), len(buf), ctypes.byref(n)), self._h)
        return buf[: n.value].tobytes()

    def redis_len(self) -> int:
        n = ctypes.c_uint64(0)
        _check(self._lib.bf_export_redis(self.handle, None, 0, ctypes.byref(n)), self._h)
        return n.value

    def import_redis(self, data: bytes, mode: int = BF_IMPORT_REPLACE) -> None:
        buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
        _check(self._lib.bf_import_redis(self.handle, _ptr(buf), len(data), int(mode)), self._h)

    # -- incremental Redis sync
    def track_dirty(self, enable: bool = True) -> None:
        """Record which BF_DIRTY_BLOCK_BYTES blocks of the Redis string inserts change."""
        _check(self._lib.bf_track_dirty(self.handle, 1 if enable else 0), self._h)

    def dirty_ranges(self, clear: bool = True) -> Tuple[List[Tuple[int, int]], int]:
        """([(byte offset, length), ...], Redis string length) changed since the last clear."""
        n, rl = ctypes.c_uint32(), ctypes.c_uint64()
        _check(self._lib.bf_dirty_ranges(self.handle, None, 0, ctypes.byref(n), ctypes.byref(rl), 0), self._h)
        while True:
            cap = max(n.value, 1)
            buf = np.zeros(2 * cap, np.uint64)
            rc = self._lib.bf_dirty_ranges(self.handle, buf.ctypes.data_as(_u64p), cap, ctypes.byref(n),
                                           ctypes.byref(rl), 1 if clear else 0)
            if rc == BF_ERANGE and n.value > cap:   # an insert on another thread grew the set
                continue
            _check(rc, self._h)
            pairs = buf[: 2 * n.value].reshape(-1, 2)
            return [(int(o), int(l)) for o, l in pairs], int(rl.value)

    def export_range(self, offset: int, length: int) -> bytes:
        buf = np.zeros(max(int(length), 1), np.uint8)
        _check(self._lib.bf_export_range(self.handle, int(offset), int(length), _ptr(buf)), self._h)
        return buf[: int(length)].tobytes()

    # -- device-resident API
    def insert_many_dev(self, d_keys: int, d_offsets: int, n: int, d_any_new: int = 0,
                        d_per_key_new: int = 0, stream=None) -> None:
        _check(self._lib.bf_insert_many_dev(self.handle, d_keys, d_offsets, int(n), d_any_new or None,
                                            d_per_key_new or None, self._s(stream)), self._h)

    def include_many_dev(self, d_keys: int, d_offsets: int, n: int, d_out: int, stream=None) -> None:
        _check(self._lib.bf_include_many_dev(self.handle, d_keys, d_offsets, int(n), d_out,
                                             self._s(stream)), self._h)

    def indexes_many_dev(self, d_keys: int, d_offsets: int, n: int, d_out: int, stream=None) -> None:
        _check(self._lib.bf_indexes_many_dev(self.handle, d_keys, d_offsets, int(n), d_out,
                                             self._s(stream)), self._h)

    # -- SHA-1 words as an intermediate (digests: 4 uint32 per key, 16-byte aligned)
    def hash_many_dev(self, d_keys: int, d_offsets: int, n: int, d_digests: int, stream=None) -> None:
        _check(self._lib.bf_hash_many_dev(self.handle, d_keys, d_offsets, int(n), d_digests, self._s(stream)),
               self._h)

    def insert_digests_dev(self, d_digests: int, n: int, d_any_new: int = 0, stream=None) -> None:
        _check(self._lib.bf_insert_digests_dev(self.handle, d_digests, int(n), d_any_new or None, None,
                                               self._s(stream)), self._h)

    def include_digests_dev(self, d_digests: int, n: int, d_out: int, stream=None) -> None:
        _check(self._lib.bf_include_digests_dev(self.handle, d_digests, int(n), d_out, self._s(stream)), self._h)

    def include_hash_dev(self, d_keys: int, d_offsets: int, n: int, d_out: int, d_next_keys: int,
                         d_next_offsets: int, n_next: int, d_next_digests: int, stream=None) -> None:
        _check(self._lib.bf_include_hash_dev(self.handle, d_keys, d_offsets, int(n), d_out, d_next_keys or None,
                                             d_next_offsets or None, int(n_next), d_next_digests or None,
                                             self._s(stream)), self._h)

    # -- replicated inserts from region sets (include/bfhip.h): encode once per rank, OR in everywhere
    def region_sets_capacity(self, n: int) -> int:
        """Bytes a region-set buffer needs for any batch of <= n keys (the same on every
        handle of this m and k)."""
        b = ctypes.c_uint64()
        _check(self._lib.bf_region_sets_capacity(self.handle, int(n), ctypes.byref(b)), self._h)
        return int(b.value)

    def encode_region_sets_dev(self, d_keys: int, d_offsets: int, n: int, d_sets: int, sets_bytes: int,
                               stream=None) -> None:
        _check(self._lib.bf_encode_region_sets_dev(self.handle, d_keys or None, d_offsets or None, int(n), d_sets,
                                                   int(sets_bytes), self._s(stream)), self._h)

    def encode_region_sets_digests_dev(self, d_digests: int, n: int, d_sets: int, sets_bytes: int,
                                       stream=None) -> None:
        _check(self._lib.bf_encode_region_sets_digests_dev(self.handle, d_digests or None, int(n), d_sets,
                                                           int(sets_bytes), self._s(stream)), self._h)

    def insert_region_sets_dev(self, d_sets: int, stride_bytes: int, nsrc: int, probes_hint: int,
                               d_any_new: int = 0, d_status: int = 0, stream=None) -> None:
        _check(self._lib.bf_insert_region_sets_dev(self.handle, d_sets, int(stride_bytes), int(nsrc),
                                                   int(probes_hint), d_any_new or None, d_status or None,
                                                   self._s(stream)), self._h)

    def insert_encode_region_sets_dev(self, d_sets: int, stride_bytes: int, nsrc: int, probes_hint: int,
                                      d_next_digests: int, n_next: int, d_next_sets: int, next_sets_bytes: int,
                                      d_any_new: int = 0, d_status: int = 0, stream=None) -> None:
        """insert_region_sets_dev of nsrc buffers and encode_region_sets_digests_dev of the next
        batch's words into d_next_sets, in one pass over the regions
        (bf_insert_encode_region_sets_dev)."""
        _check(self._lib.bf_insert_encode_region_sets_dev(self.handle, d_sets or None, int(stride_bytes), int(nsrc),
                                                          int(probes_hint), d_any_new or None, d_status or None,
                                                          d_next_digests or None, int(n_next), d_next_sets,
                                                          int(next_sets_bytes), self._s(stream)), self._h)

    def _s(self, stream):
        if stream is None:
            if getattr(self, "_own_stream", None) is None:
                p = _vp()
                _check(self._lib.bf_stream(self.handle, ctypes.byref(p)), self._h)
                self._own_stream = p.value or 0
            return self._own_stream or None
        return int(stream) or None

    def insert_plan(self, n: int) -> dict:
        """How an insert of n keys runs: {"binned": bool, "scratch_bytes": int} (bf_insert_plan)."""
        b, sb = ctypes.c_uint32(), ctypes.c_uint64()
        _check(self._lib.bf_insert_plan(self.handle, int(n), ctypes.byref(b), ctypes.byref(sb)), self._h)
        return {"binned": bool(b.value), "scratch_bytes": int(sb.value)}

    def profile(self, enable: bool) -> None:
        """Per-kernel HIP-event timing of every keyed launch (bf_profile)."""
        _check(self._lib.bf_profile(self.handle, 1 if enable else 0), self._h)

    def profile_read(self, reset: bool = True) -> dict:
        """{kernel name: (total ms, launches)} since the last reset (bf_profile_read)."""
        cap = 32
        names = ctypes.create_string_buffer(cap * PROFILE_NAME_LEN)
        ms = np.zeros(cap, np.float64)
        cnt = np.zeros(cap, np.uint64)
        n = ctypes.c_uint32()
        _check(self._lib.bf_profile_read(self.handle, names, _ptr(ms), _ptr(cnt), cap, ctypes.byref(n),
                                         1 if reset else 0), self._h)
        out = {}
        for i in range(min(n.value, cap)):
            raw = names.raw[i * PROFILE_NAME_LEN:(i + 1) * PROFILE_NAME_LEN]
            out[raw.split(b"\0", 1)[0].decode()] = (float(ms[i]), int(cnt[i]))
        return out

    def device_bits(self) -> Tuple[int, int]:
        p = _vp()
        nb = ctypes.c_uint64()
        _check(self._lib.bf_device_bits(self.handle, ctypes.byref(p), ctypes.byref(nb)), self._h)
        return int(p.value or 0), int(nb.value)

    # -- partitioned filters (see include/bfhip.h)
    def route_dev(self, d_keys: int, d_offsets: int, n: int, d_send: int, d_slot: int, d_counts: int,
                  stream=None) -> None:
        _check(self._lib.bf_route_dev(self.handle, d_keys, d_offsets, int(n), d_send, d_slot or None, d_counts,
                                      self._s(stream)), self._h)

    def route_windows_dev(self, d_keys: int, d_offsets: int, n: int, d_send: int, d_slot: int, window_cap: int,
                          d_counts: int, stream=None) -> None:
        _check(self._lib.bf_route_windows_dev(self.handle, d_keys, d_offsets, int(n), d_send, d_slot or None,
                                              int(window_cap), d_counts, self._s(stream)), self._h)

    def route_window_split(self) -> int:
        nh = ctypes.c_uint32()
        _check(self._lib.bf_route_window_split(self.handle, ctypes.byref(nh)), self._h)
        return int(nh.value)

    # -- chunked windows (the owner skips its sort pass; include/bfhip.h)
    def route_chunk_info(self, n_bound: int):
        """(tiles, dir_bytes, superbins per window) for batches of <= n_bound keys, or None
        when this shard count cannot take chunked windows."""
        t, d, sb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
        if self._lib.bf_route_chunk_info(self.handle, int(n_bound), ctypes.byref(t), ctypes.byref(d),
                                         ctypes.byref(sb)) != 0:
            return None
        return int(t.value), int(d.value), int(sb.value)

    def route_chunks_dev(self, d_keys: int, d_offsets: int, n: int, d_send: int, d_slot16: int, window_cap: int,
                         d_counts: int, d_dir: int, dir_bytes: int, tiles: int, stream=None) -> None:
        _check(self._lib.bf_route_chunks_dev(self.handle, d_keys, d_offsets, int(n), d_send, d_slot16 or None,
                                             int(window_cap), d_counts, d_dir, int(dir_bytes), int(tiles),
                                             self._s(stream)), self._h)

    def route_chunks_digests_dev(self, d_digests: int, n: int, d_send: int, d_slot16: int, window_cap: int,
                                 d_counts: int, d_dir: int, dir_bytes: int, tiles: int, stream=None) -> None:
        """route_chunks_dev from the keys' SHA-1 words (hash_many_dev's output)."""
        _check(self._lib.bf_route_chunks_digests_dev(self.handle, d_digests, int(n), d_send, d_slot16 or None,
                                                     int(window_cap), d_counts, d_dir, int(dir_bytes), int(tiles),
                                                     self._s(stream)), self._h)

    def shard_insert_chunks_dev(self, d_recv: int, window_cap: int, nsrc: int, d_dir: int, dir_bytes: int, tiles: int,
                                d_counts: int, count_stride: int, d_any_new: int = 0, stream=None) -> None:
        _check(self._lib.bf_shard_insert_chunks_dev(self.handle, d_recv, int(window_cap), int(nsrc), d_dir,
                                                    int(dir_bytes), int(tiles), d_counts, int(count_stride),
                                                    d_any_new or None, self._s(stream)), self._h)

    def shard_test_chunks_dev(self, d_recv: int, window_cap: int, nsrc: int, d_dir: int, dir_bytes: int, tiles: int,
                              d_counts: int, count_stride: int, d_bits: int, stream=None) -> None:
        _check(self._lib.bf_shard_test_chunks_dev(self.handle, d_recv, int(window_cap), int(nsrc), d_dir,
                                                  int(dir_bytes), int(tiles), d_counts, int(count_stride), d_bits,
                                                  self._s(stream)), self._h)

    def shard_test_chunks_packed_dev(self, d_recv: int, window_cap: int, nsrc: int, d_dir: int, dir_bytes: int,
                                     tiles: int, d_counts: int, count_stride: int, d_packed: int, stream=None) -> None:
        """The owner test with its answers as packed bits in the return trip's layout (window
        (hi, src) at d_packed + (src * nh + hi) * ceil(window_cap / 8))."""
        _check(self._lib.bf_shard_test_chunks_packed_dev(self.handle, d_recv, int(window_cap), int(nsrc), d_dir,
                                                         int(dir_bytes), int(tiles), d_counts, int(count_stride),
                                                         d_packed, self._s(stream)), self._h)

    def shard_insert_test_chunks_packed_dev(self, d_ins_recv: int, d_ins_dir: int, d_ins_counts: int,
                                            d_tst_recv: int, d_tst_dir: int, d_tst_counts: int, window_cap: int,
                                            nsrc: int, dir_bytes: int, tiles: int, count_stride: int,
                                            d_packed: int, d_any_new: int = 0, d_next_keys: int = 0,
                                            d_next_offsets: int = 0, n_next: int = 0, d_next_digests: int = 0,
                                            stream=None) -> None:
        """One step's owner work: the insert windows ORed in, then the include? windows tested
        (packed answers as shard_test_chunks_packed_dev), in one pass over the shard; with
        n_next, that pass also hashes another key batch into d_next_digests."""
        _check(self._lib.bf_shard_insert_test_chunks_packed_dev(
            self.handle, d_ins_recv, d_ins_dir, d_ins_counts, d_tst_recv, d_tst_dir, d_tst_counts, int(window_cap),
            int(nsrc), int(dir_bytes), int(tiles), int(count_stride), d_any_new or None, d_packed,
            d_next_keys or None, d_next_offsets or None, int(n_next), d_next_digests or None,
            self._s(stream)), self._h)

    def shard_test_chunks_hash_dev(self, d_recv: int, window_cap: int, nsrc: int, d_dir: int, dir_bytes: int,
                                   tiles: int, d_counts: int, count_stride: int, d_bits: int, d_next_keys: int,
                                   d_next_offsets: int, n_next: int, d_next_digests: int, stream=None) -> None:
        """shard_test_chunks_dev that also hashes another key batch (SHA-1 words to d_next_digests)."""
        _check(self._lib.bf_shard_test_chunks_hash_dev(self.handle, d_recv, int(window_cap), int(nsrc), d_dir,
                                                       int(dir_bytes), int(tiles), d_counts, int(count_stride), d_bits,
                                                       d_next_keys or None, d_next_offsets or None, int(n_next),
                                                       d_next_digests or None, self._s(stream)), self._h)

    def combine_chunks_packed_dev(self, d_packed: int, d_slot16: int, window_cap: int, d_dir: int, dir_bytes: int,
                                  tiles: int, d_counts: int, n: int, d_out: int, stream=None) -> None:
        _check(self._lib.bf_combine_chunks_packed_dev(self.handle, d_packed, d_slot16, int(window_cap), d_dir,
                                                      int(dir_bytes), int(tiles), d_counts, int(n), d_out,
                                                      self._s(stream)), self._h)

    def pack_segments_dev(self, d_bits: int, d_seg: int, nseg: int, max_count: int, d_packed: int,
                          stream=None) -> None:
        _check(self._lib.bf_pack_segments_dev(self.handle, d_bits, d_seg, int(nseg), int(max_count), d_packed,
                                              self._s(stream)), self._h)

    def combine_windows_packed_dev(self, d_packed: int, d_slot: int, window_cap: int, nwin: int, d_counts: int,
                                   n: int, d_out: int, stream=None) -> None:
        _check(self._lib.bf_combine_windows_packed_dev(self.handle, d_packed, d_slot, int(window_cap), int(nwin),
                                                       d_counts, int(n), d_out, self._s(stream)), self._h)

    def shard_insert_windows_dev(self, d_local32: int, window_cap: int, nwin: int, d_counts: int, count_stride: int,
                                 hi: int, d_any_new: int = 0, stream=None) -> None:
        _check(self._lib.bf_shard_insert_windows_dev(self.handle, d_local32, int(window_cap), int(nwin), d_counts,
                                                     int(count_stride), int(hi), d_any_new or None, self._s(stream)),
               self._h)

    def shard_test_windows_dev(self, d_local32: int, window_cap: int, nwin: int, d_counts: int, count_stride: int,
                               hi: int, d_bits: int, stream=None) -> None:
        _check(self._lib.bf_shard_test_windows_dev(self.handle, d_local32, int(window_cap), int(nwin), d_counts,
                                                   int(count_stride), int(hi), d_bits, self._s(stream)), self._h)

    def shard_insert_hi_dev(self, d_local32: int, count: int, hi: int, d_any_new: int = 0, stream=None) -> None:
        _check(self._lib.bf_shard_insert_hi_dev(self.handle, d_local32, int(count), int(hi), d_any_new or None,
                                                self._s(stream)), self._h)

    def shard_test_hi_dev(self, d_local32: int, count: int, hi: int, d_bits: int, stream=None) -> None:
        _check(self._lib.bf_shard_test_hi_dev(self.handle, d_local32, int(count), int(hi), d_bits, self._s(stream)),
               self._h)

    def combine_windows_dev(self, d_bits: int, d_slot: int, window_cap: int, nwin: int, d_counts: int, n: int,
                            d_out: int, stream=None) -> None:
        _check(self._lib.bf_combine_windows_dev(self.handle, d_bits, d_slot, int(window_cap), int(nwin), d_counts,
                                                int(n), d_out, self._s(stream)), self._h)

    def shard_insert_dev(self, d_local: int, count: int, d_any_new: int = 0, stream=None) -> None:
        _check(self._lib.bf_shard_insert_dev(self.handle, d_local, int(count), d_any_new or None,
                                             self._s(stream)), self._h)

    def shard_test_dev(self, d_local: int, count: int, d_bits: int, stream=None) -> None:
        _check(self._lib.bf_shard_test_dev(self.handle, d_local, int(count), d_bits, self._s(stream)), self._h)

    def combine_dev(self, d_bits: int, d_slot: int, n: int, d_out: int, stream=None) -> None:
        _check(self._lib.bf_combine_dev(self.handle, d_bits, d_slot, int(n), d_out, self._s(stream)), self._h)

    def shard_export(self) -> np.ndarray:
        n = ctypes.c_uint64(0)
        _check(self._lib.bf_shard_export(self.handle, None, 0, ctypes.byref(n)), self._h)
        buf = np.zeros(max(n.value, 1), np.uint8)
        _check(self._lib.bf_shard_export(self.handle, _ptr(buf), len(buf), ctypes.byref(n)), self._h)
        return buf[: n.value]

    def shard_import(self, data, mode: int = BF_IMPORT_REPLACE) -> None:
        buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
        _check(self._lib.bf_shard_import(self.handle, _ptr(buf), len(buf) if len(data) else 0, int(mode)),
               self._h)


def lua_layer_params(entries, precision, layer: int) -> Tuple[int, int]:
    """(bits, k) of layer `layer` of the Lua scalable filter (add.lua:16-25)."""
    b, k = ctypes.c_uint64(), ctypes.c_uint32()
    rc = load().bf_lua_layer_params(float(entries), float(precision), int(layer), ctypes.byref(b), ctypes.byref(k))
    if rc:
        raise ArgumentError("bf_lua_layer_params(%r, %r, %r) failed" % (entries, precision, layer))
    return int(b.value), int(k.value)


def lua_index(entries, count: int) -> int:
    """The layer a count maps to (add.lua:13-15 / check.lua:9-11)."""
    li = ctypes.c_uint32()
    if load().bf_lua_index(float(entries), int(count), ctypes.byref(li)):
        raise ArgumentError("bf_lua_index(%r, %r) failed" % (entries, count))
    return int(li.value)


def _lua_check(code: int, h=None) -> None:
    if code == BF_OK:
        return
    msg = load().bf_lua_last_error(h).decode(errors="replace")
    if code in (BF_EINVAL, BF_ERANGE):
        raise ArgumentError("%s: %s" % (_STATUS.get(code), msg))
    raise BfHipError(code, msg)


class LuaFilter:
    """The Lua driver's scalable filter on the device (a ``bf_lua*``; see include/bfhip.h)."""

    def __init__(self, entries, precision, device: int = -1):
        self._lib = load()
        cfg = bf_config(ctypes.sizeof(bf_config), int(device), 0, 0, 1, 0, 0, 0)
        h = _vp()
        _lua_check(self._lib.bf_lua_create(float(entries), float(precision), ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.entries, self.precision = entries, precision

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.bf_lua_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        if not self._h:
            raise ArgumentError("filter is closed")
        return self._h

    def insert_many(self, keys: np.ndarray, offsets: np.ndarray):
        """-> (per-key new flags, sorted list of layers that got a new item)."""
        keys, offsets, n = Filter._keys(keys, offsets)
        pk = np.zeros(max(n, 1), np.uint8)
        mask = ctypes.c_uint64(0)
        _lua_check(self._lib.bf_lua_insert_many(self.handle, _ptr(keys), _ptr(offsets), n, _ptr(pk),
                                                ctypes.byref(mask)), self._h)
        return pk[:n], [i + 1 for i in range(64) if mask.value >> i & 1]

    LAYER_SHIFT = 58   # BF_LUA_LAYER_SHIFT

    def insert_many_changes(self, keys: np.ndarray, offsets: np.ndarray):
        """-> (per-key new flags, layers that got a new item, [(layer, bit offset), ...] of every
        bit the batch flipped, each once: the SETBITs add.lua issued that changed something)."""
        keys, offsets, n = Filter._keys(keys, offsets)
        pk = np.zeros(max(n, 1), np.uint8)
        mask = ctypes.c_uint64(0)
        cap = max(64 * n, 1)   # BF_MAX_K probes per key at most
        out = np.zeros(cap, np.uint64)
        cnt = ctypes.c_uint64(0)
        _lua_check(self._lib.bf_lua_insert_many_changes(self.handle, _ptr(keys), _ptr(offsets), n, _ptr(pk),
                                                        ctypes.byref(mask), _ptr(out), cap, ctypes.byref(cnt)),
                   self._h)
        flips = out[: cnt.value]
        sh = np.uint64(self.LAYER_SHIFT)
        pairs = list(zip((flips >> sh).tolist(), (flips & ((np.uint64(1) << sh) - np.uint64(1))).tolist()))
        return pk[:n], [i + 1 for i in range(64) if mask.value >> i & 1], pairs

    def include_many(self, keys: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        keys, offsets, n = Filter._keys(keys, offsets)
        out = np.zeros(max(n, 1), np.uint8)
        _lua_check(self._lib.bf_lua_include_many(self.handle, _ptr(keys), _ptr(offsets), n, _ptr(out)), self._h)
        return out[:n]

    # -- device-resident keys (bf_lua_insert_many_dev / bf_lua_include_many_dev): raw device
    #    addresses and a hipStream_t as ints, as Filter's *_dev methods
    def insert_many_dev(self, d_keys: int, d_offsets: int, n: int, d_per_key_new: int = 0, stream=0) -> list:
        """add.lua over n device keys; returns the layers that got a new item."""
        mask = ctypes.c_uint64()
        _lua_check(self._lib.bf_lua_insert_many_dev(self.handle, d_keys, d_offsets, int(n), d_per_key_new or None,
                                                    ctypes.byref(mask), int(stream) or None), self._h)
        return [i + 1 for i in range(64) if mask.value >> i & 1]

    def include_many_dev(self, d_keys: int, d_offsets: int, n: int, d_out: int, stream=0) -> None:
        _lua_check(self._lib.bf_lua_include_many_dev(self.handle, d_keys, d_offsets, int(n), d_out,
                                                     int(stream) or None), self._h)

    def profile(self, enable: bool) -> None:
        _lua_check(self._lib.bf_lua_profile(self.handle, 1 if enable else 0), self._h)

    def profile_read(self, reset: bool = True) -> dict:
        """{kernel name: (total ms, launches)} since the last reset (bf_lua_profile_read)."""
        cap = 64
        names = ctypes.create_string_buffer(cap * PROFILE_NAME_LEN)
        ms = np.zeros(cap, np.float64)
        cnt = np.zeros(cap, np.uint64)
        n = ctypes.c_uint32()
        _lua_check(self._lib.bf_lua_profile_read(self.handle, names, _ptr(ms), _ptr(cnt), cap, ctypes.byref(n),
                                                 1 if reset else 0), self._h)
        out = {}
        for i in range(min(n.value, cap)):
            raw = names.raw[i * PROFILE_NAME_LEN:(i + 1) * PROFILE_NAME_LEN]
            out[raw.split(b"\0", 1)[0].decode()] = (float(ms[i]), int(cnt[i]))
        return out

    def clear(self) -> None:
        _lua_check(self._lib.bf_lua_clear(self.handle), self._h)

    @property
    def count(self) -> int:
        c = ctypes.c_uint64()
        _lua_check(self._lib.bf_lua_get_count(self.handle, ctypes.byref(c)), self._h)
        return int(c.value)

    @count.setter
    def count(self, value: int) -> None:
        _lua_check(self._lib.bf_lua_set_count(self.handle, int(value)), self._h)

    @property
    def layers(self) -> int:
        n = ctypes.c_uint32()
        _lua_check(self._lib.bf_lua_layers(self.handle, ctypes.byref(n)), self._h)
        return int(n.value)

    def export_layer(self, layer: int) -> bytes:
        n = ctypes.c_uint64(0)
        _lua_check(self._lib.bf_lua_export_layer(self.handle, int(layer), None, 0, ctypes.byref(n)), self._h)
        buf = np.zeros(max(n.value, 1), np.uint8)
        _lua_check(self._lib.bf_lua_export_layer(self.handle, int(layer), _ptr(buf), len(buf), ctypes.byref(n)),
                   self._h)
        return buf[: n.value].tobytes()

    def import_layer(self, layer: int, data: bytes) -> None:
        buf = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
        _lua_check(self._lib.bf_lua_import_layer(self.handle, int(layer), _ptr(buf), len(data)), self._h)
