"""Multi-GPU filters: one process per GPU, collectives through torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests and, with device
tensors staged through host memory, for several ranks sharing one GPU in the GPU tests).

Two layouts (SURVEY §8 e):

``PartitionedFilter`` — the filter's reachable prefix is split block-cyclically
    over the P ranks (block = 2^block_log2 bits, owner = block % P), so a
    filter larger than one GPU's HBM (the 200B-key config) fits, and the
    probe-dense low offsets (h0 < 2^32, ruby.rb:51) spread over every GPU.
    insert:   route (hash -> owner-local offsets, one send window per owner) ->
              all_to_all(counts) -> all_to_all(offsets) -> owner OR
    include?: route -> all_to_all(offsets) -> owner bit test ->
              reverse all_to_all(1 byte per probe) -> requester AND per key
    Each rank brings its own key batch (weak scaling); the only data-path
    collectives are the two all-to-alls the ownership split makes necessary.

``ReplicatedFilter`` — every rank holds the whole filter (read-mostly
    filters that fit one GPU).  include? is purely local (no collective);
    insert all-gathers the key bytes and key lengths (one byte per key while
    keys fit 255 bytes) beside the rank's own insert, then applies the other
    ranks' batches as one insert, so the replicas stay byte-identical.

The per-rank compute goes through an *engine* with four primitives (route,
shard_insert, shard_test, combine) plus the window forms of route and combine;
``HipEngine`` is libbfhip.so's ``bf_route[_windows]_dev`` / ``bf_shard_*_dev`` /
``bf_combine[_windows]_dev``.  The all-to-alls are grouped sends/receives
(``batch_isend_irecv``: one RCCL group of ncclSend/ncclRecv), so each owner's
segment can sit in its own window of the send buffer.  The CPU tests
substitute a numpy engine to exercise this module's exchange logic over gloo.
"""
from __future__ import annotations

import os
import time
from typing import Iterable, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import keys as _keys
from ._lib import BF_EINVAL, BF_FLAG_ENCODER, BF_FLAG_ROUTE32, ArgumentError, BfHipError, Filter

# -- collectives -------------------------------------------------------------------------
# RCCL (backend "nccl") moves device tensors directly.  Under gloo the device tensors are
# staged through host memory (synchronously: the returned works are already complete), so
# the same exchange runs over gloo with several ranks sharing one GPU — the multi-rank
# rehearsal of the HIP engine on a one-GPU box (tests/test_gpu_dist_gloo.py), where RCCL
# refuses a communicator whose ranks share a device.


class _Done:
    """A completed work handle (host-staged collectives finish before they return)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == dist.Backend.GLOO


def _all_to_all_single(recv: torch.Tensor, send: torch.Tensor, group=None, async_op: bool = False):
    if not _staged(recv, group):
        return dist.all_to_all_single(recv, send, group=group, async_op=async_op)
    host = torch.empty(recv.shape, dtype=recv.dtype)
    dist.all_to_all_single(host, send.cpu(), group=group)
    recv.copy_(host)
    return _Done() if async_op else None


def _all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor, group=None, async_op: bool = False):
    if not _staged(out, group):
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    host = torch.empty(out.shape, dtype=out.dtype)
    dist.all_gather_into_tensor(host, inp.cpu(), group=group)
    out.copy_(host)
    return _Done() if async_op else None


def _all_reduce(t: torch.Tensor, op, group=None) -> None:
    if not _staged(t, group):
        dist.all_reduce(t, op=op, group=group)
        return
    host = t.cpu()
    dist.all_reduce(host, op=op, group=group)
    t.copy_(host)


def _send(t: torch.Tensor, dst: int, group=None) -> None:
    dist.send(t.cpu() if _staged(t, group) else t, dst, group=group)


def _recv(t: torch.Tensor, src: int, group=None) -> None:
    if not _staged(t, group):
        dist.recv(t, src, group=group)
        return
    host = torch.empty(t.shape, dtype=t.dtype)
    dist.recv(host, src, group=group)
    t.copy_(host)


def _batch_p2p(sends, recvs, group=None):
    """sends / recvs: [(global peer, tensor)]; one group of isend/irecv (messages between two
    ranks match in list order).  Returns the works to wait on."""
    ref = sends[0][1] if sends else (recvs[0][1] if recvs else None)
    if ref is None:
        return []
    if not _staged(ref, group):
        ops = [dist.P2POp(dist.isend, t, g, group) for g, t in sends]
        ops += [dist.P2POp(dist.irecv, t, g, group) for g, t in recvs]
        return dist.batch_isend_irecv(ops)
    hs = [(g, t.cpu()) for g, t in sends]
    hr = [(g, torch.empty(t.shape, dtype=t.dtype)) for g, t in recvs]
    ops = [dist.P2POp(dist.isend, t, g, group) for g, t in hs]
    ops += [dist.P2POp(dist.irecv, t, g, group) for g, t in hr]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    for (_, t), (_, h) in zip(recvs, hr):
        t.copy_(h)
    return [_Done()]


def block_owner_local(offsets: np.ndarray, P: int, block_log2: int) -> Tuple[np.ndarray, np.ndarray]:
    """Host restatement of the ownership map in include/bfhip.h (for tooling and tests)."""
    o = offsets.astype(np.uint64)
    blk = o >> np.uint64(block_log2)
    owner = (blk % np.uint64(P)).astype(np.int64)
    local = ((blk // np.uint64(P)) << np.uint64(block_log2)) | (o & np.uint64((1 << block_log2) - 1))
    return owner, local


def shard_local_bits(reach_bits: int, P: int, s: int, block_log2: int) -> int:
    nblocks = (reach_bits + (1 << block_log2) - 1) >> block_log2
    mine = (nblocks - 1 - s) // P + 1 if nblocks > s else 0
    return mine << block_log2


def interleave_shards(shards: List[np.ndarray], reach_bits: int, block_log2: int) -> bytes:
    """Rebuild the Redis string (trimmed) from every shard's local bytes."""
    P = len(shards)
    bb = (1 << block_log2) // 8
    nblocks = (reach_bits + (1 << block_log2) - 1) >> block_log2
    out = np.zeros(nblocks * bb, dtype=np.uint8)
    view = out.reshape(nblocks, bb)
    for s, loc in enumerate(shards):
        cnt = len(range(s, nblocks, P))
        if cnt:
            arr = np.asarray(loc, dtype=np.uint8)[: cnt * bb]
            if len(arr) < cnt * bb:   # a whole-filter handle (P == 1) stops at the reachable prefix
                arr = np.concatenate([arr, np.zeros(cnt * bb - len(arr), np.uint8)])
            view[s::P] = arr.reshape(cnt, bb)
    out = out[: (reach_bits + 7) // 8]
    nz = np.flatnonzero(out)
    return out[: nz[-1] + 1].tobytes() if len(nz) else b""


def split_shard(data: bytes, P: int, s: int, reach_bits: int, block_log2: int) -> np.ndarray:
    """Shard s's local bytes of a Redis string (inverse of interleave_shards)."""
    bb = (1 << block_log2) // 8
    nblocks = (reach_bits + (1 << block_log2) - 1) >> block_log2
    full = np.zeros(nblocks * bb, dtype=np.uint8)
    src = np.frombuffer(data, dtype=np.uint8)
    if len(src) > (reach_bits + 7) // 8:
        raise ArgumentError("string of %d bytes exceeds the filter's reachable bytes" % len(src))
    full[: len(src)] = src
    return np.ascontiguousarray(full.reshape(nblocks, bb)[s::P]).reshape(-1)


class HipEngine:
    """Per-rank primitives on libbfhip.so (one shard handle on this rank's GPU)."""

    def __init__(self, m: int, k: int, P: int, rank: int, block_log2: int, device: torch.device):
        self.device = device
        reach = min(m, k * 0xFFFFFFFF + 1)
        # 32-bit owner-local offsets halve the all-to-all bytes whenever every shard fits 2^32 bits
        route32 = shard_local_bits(reach, P, 0, block_log2) <= (1 << 32)
        self.filter = Filter(m, k, device=device.index if device.index is not None else -1,
                             shard_count=P, shard_index=rank, shard_block_log2=block_log2,
                             flags=BF_FLAG_ROUTE32 if route32 else 0)
        self.k, self.P = k, P
        self.offset_dtype = torch.int32 if route32 else torch.int64
        self.nh = self.filter.route_window_split()   # 2^32-bit sub-ranges per window-routed owner
        # Test hook (PartitionedFilter(poison=...) / BFHIP_POISON_WINDOWS): the route's send
        # windows and slots are filled before the route writes them, so an owner or combine
        # that reads an entry past a window's live count reads a known wrong value instead of
        # whatever the caching allocator handed back (the r02 illegal-address fault).
        self.poison = None

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def route(self, kb: torch.Tensor, ko: torch.Tensor, n: int, want_slot: bool = True):
        """Probes grouped by owner (send), per-owner counts, and (for include?) the key
        index of every send entry (slot)."""
        send = torch.empty(n * self.k, dtype=self.offset_dtype, device=self.device)
        slot = torch.empty(n * self.k, dtype=torch.int32, device=self.device) if want_slot else None
        counts = torch.empty(self.P, dtype=torch.int64, device=self.device)
        self.filter.route_dev(kb.data_ptr(), ko.data_ptr(), n, send.data_ptr(),
                              slot.data_ptr() if want_slot else 0, counts.data_ptr(), stream=self._stream())
        return send, slot, counts

    def route_windows(self, kb: torch.Tensor, ko: torch.Tensor, n: int, cap: int, want_slot: bool = True):
        """route() without the owner-major gather: window w = owner * nh + hi holds that owner's
        probes with local offset (hi << 32) | entry, as uint32, in send[w*cap : w*cap +
        counts[w]] in an unspecified order (slot alongside); counts[w] > cap = overflow."""
        nwin = self.P * self.nh
        send = torch.empty(nwin * cap, dtype=torch.int32, device=self.device)
        slot = torch.empty(nwin * cap, dtype=torch.int32, device=self.device) if want_slot else None
        counts = torch.empty(nwin, dtype=torch.int64, device=self.device)
        if self.poison is not None:
            send.fill_(self.poison)
            if slot is not None:
                slot.fill_(0)   # a dead slot names key 0: a stray AND into it shows as a wrong answer
        self.filter.route_windows_dev(kb.data_ptr(), ko.data_ptr(), n, send.data_ptr(),
                                      slot.data_ptr() if want_slot else 0, cap, counts.data_ptr(),
                                      stream=self._stream())
        return send, slot, counts

    # -- chunked windows: the owner's sort pass moves into the route (include/bfhip.h)
    def chunk_info(self, n_bound: int):
        """(tiles, dir_bytes) of the chunk directories for batches of <= n_bound keys (the same
        on every rank), or None when this shard count cannot take chunked windows."""
        info = self.filter.route_chunk_info(n_bound)
        return info[:2] if info else None

    def route_chunks(self, kb: torch.Tensor, ko: torch.Tensor, n: int, cap: int, tiles: int, dir_bytes: int,
                     want_slot: bool = True):
        """route_windows whose per-tile runs are sorted by owner superbin, plus one directory
        per window (dir_bytes each) and tile-relative uint16 slots."""
        nwin = self.P * self.nh
        send = torch.empty(nwin * cap, dtype=torch.int32, device=self.device)
        slot = torch.empty(nwin * cap, dtype=torch.int16, device=self.device) if want_slot else None
        counts = torch.empty(nwin, dtype=torch.int64, device=self.device)
        dirb = torch.empty(nwin * dir_bytes, dtype=torch.uint8, device=self.device)
        if self.poison is not None:
            send.fill_(self.poison)
            if slot is not None:
                slot.fill_(0)
        if kb is not None and ko is None:   # kb: the keys' SHA-1 words (hash_keys / shard_test_chunks(next=))
            self.filter.route_chunks_digests_dev(kb.data_ptr(), n, send.data_ptr(), slot.data_ptr() if want_slot else 0,
                                                 cap, counts.data_ptr(), dirb.data_ptr(), dir_bytes, tiles,
                                                 stream=self._stream())
        else:
            self.filter.route_chunks_dev(kb.data_ptr(), ko.data_ptr(), n, send.data_ptr(),
                                         slot.data_ptr() if want_slot else 0, cap, counts.data_ptr(), dirb.data_ptr(),
                                         dir_bytes, tiles, stream=self._stream())
        return send, slot, counts, dirb

    def hash_keys(self, kb: torch.Tensor, ko: torch.Tensor, n: int, out: torch.Tensor = None) -> torch.Tensor:
        """The keys' SHA-1 words (n x 4 int32), route_chunks' digest input."""
        dig = out if out is not None else torch.empty((max(n, 1), 4), dtype=torch.int32, device=self.device)
        if n:
            self.filter.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n, dig.data_ptr(), stream=self._stream())
        return dig

    def shard_insert_chunks(self, recv: torch.Tensor, cap: int, nsrc: int, rdir: torch.Tensor, dir_bytes: int,
                            tiles: int, counts: torch.Tensor, cstride: int) -> None:
        """OR every sub-range's received chunked windows (window (h, src) at (h*nsrc + src)*cap,
        live count counts.view(-1)[src*cstride + h]) in one call."""
        self.filter.shard_insert_chunks_dev(recv.data_ptr(), cap, nsrc, rdir.data_ptr(), dir_bytes, tiles,
                                            counts.data_ptr(), cstride, stream=self._stream())

    def shard_test_chunks(self, recv: torch.Tensor, cap: int, nsrc: int, rdir: torch.Tensor, dir_bytes: int,
                          tiles: int, counts: torch.Tensor, cstride: int, out: torch.Tensor, nxt=None) -> None:
        """nxt = (kb, ko, n, dig): the owner test's waves also hash that batch into dig (n x 4 int32)."""
        if nxt is not None and nxt[2]:
            kb, ko, n, dig = nxt
            self.filter.shard_test_chunks_hash_dev(recv.data_ptr(), cap, nsrc, rdir.data_ptr(), dir_bytes, tiles,
                                                   counts.data_ptr(), cstride, out.data_ptr(), kb.data_ptr(),
                                                   ko.data_ptr(), n, dig.data_ptr(), stream=self._stream())
            return
        self.filter.shard_test_chunks_dev(recv.data_ptr(), cap, nsrc, rdir.data_ptr(), dir_bytes, tiles,
                                          counts.data_ptr(), cstride, out.data_ptr(), stream=self._stream())

    def shard_test_chunks_packed(self, recv: torch.Tensor, cap: int, nsrc: int, rdir: torch.Tensor, dir_bytes: int,
                                 tiles: int, counts: torch.Tensor, cstride: int) -> torch.Tensor:
        """The owner test's answers as packed bits, laid out as the return trip sends them:
        window (h, src) at (src * nh + h) * ceil(cap / 8) (no pack pass)."""
        cap8 = (cap + 7) // 8
        packed = torch.empty(max(nsrc * self.nh * cap8, 1), dtype=torch.uint8, device=self.device)
        self.filter.shard_test_chunks_packed_dev(recv.data_ptr(), cap, nsrc, rdir.data_ptr(), dir_bytes, tiles,
                                                 counts.data_ptr(), cstride, packed.data_ptr(), stream=self._stream())
        return packed

    def shard_insert_test_chunks_packed(self, irecv: torch.Tensor, irdir: torch.Tensor, icounts: torch.Tensor,
                                        trecv: torch.Tensor, trdir: torch.Tensor, tcounts: torch.Tensor, cap: int,
                                        nsrc: int, dir_bytes: int, tiles: int, cstride: int, nxt=None) -> torch.Tensor:
        """shard_insert_chunks then shard_test_chunks_packed, in one pass over the shard where
        both take their sorted forms; returns the packed answers.  nxt = (kb, ko, n, dig): the
        pass also hashes that batch into dig (n x 4 int32)."""
        cap8 = (cap + 7) // 8
        packed = torch.empty(max(nsrc * self.nh * cap8, 1), dtype=torch.uint8, device=self.device)
        kb, ko, nn, dig = nxt if nxt is not None and nxt[2] else (None, None, 0, None)
        self.filter.shard_insert_test_chunks_packed_dev(irecv.data_ptr(), irdir.data_ptr(), icounts.data_ptr(),
                                                        trecv.data_ptr(), trdir.data_ptr(), tcounts.data_ptr(), cap,
                                                        nsrc, dir_bytes, tiles, cstride, packed.data_ptr(),
                                                        d_next_keys=kb.data_ptr() if nn else 0,
                                                        d_next_offsets=ko.data_ptr() if nn else 0, n_next=nn,
                                                        d_next_digests=dig.data_ptr() if nn else 0,
                                                        stream=self._stream())
        return packed

    def combine_chunks_packed(self, packed: torch.Tensor, slot: torch.Tensor, cap: int, dirb: torch.Tensor,
                              dir_bytes: int, tiles: int, counts: torch.Tensor, n: int) -> torch.Tensor:
        out = torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)[:n]
        self.filter.combine_chunks_packed_dev(packed.data_ptr(), slot.data_ptr(), cap, dirb.data_ptr(), dir_bytes,
                                              tiles, counts.data_ptr(), n, out.data_ptr(), stream=self._stream())
        return out

    def combine_windows(self, bits: torch.Tensor, slot: torch.Tensor, counts: torch.Tensor, cap: int,
                        n: int) -> torch.Tensor:
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self.filter.combine_windows_dev(bits.data_ptr(), slot.data_ptr(), cap, counts.numel(), counts.data_ptr(), n,
                                        out.data_ptr(), stream=self._stream())
        return out

    def pack_answers(self, bits: torch.Tensor, seg: torch.Tensor, max_count: int, total: int) -> torch.Tensor:
        """Answer bytes -> bits per segment (seg: [nseg, 3] int64 src, count, dst byte)."""
        packed = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
        self.filter.pack_segments_dev(bits.data_ptr(), seg.data_ptr(), seg.shape[0], max_count, packed.data_ptr(),
                                      stream=self._stream())
        return packed

    def combine_windows_packed(self, packed: torch.Tensor, slot: torch.Tensor, counts: torch.Tensor, cap: int,
                               n: int) -> torch.Tensor:
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self.filter.combine_windows_packed_dev(packed.data_ptr(), slot.data_ptr(), cap, counts.numel(),
                                               counts.data_ptr(), n, out.data_ptr(), stream=self._stream())
        return out

    def shard_insert_windows(self, recv: torch.Tensor, cap: int, nwin: int, counts: torch.Tensor, col: int,
                             stride: int, hi: int) -> None:
        """OR nwin received windows of cap uint32 entries (sub-range hi); window w's live count
        is counts.view(-1)[w * stride + col], on the device."""
        self.filter.shard_insert_windows_dev(recv.data_ptr(), cap, nwin, counts.data_ptr() + 8 * col, stride, hi,
                                             stream=self._stream())

    def shard_test_windows(self, recv: torch.Tensor, cap: int, nwin: int, counts: torch.Tensor, col: int,
                           stride: int, hi: int, out: torch.Tensor) -> None:
        self.filter.shard_test_windows_dev(recv.data_ptr(), cap, nwin, counts.data_ptr() + 8 * col, stride, hi,
                                           out.data_ptr(), stream=self._stream())

    def shard_insert_hi(self, local32: torch.Tensor, hi: int) -> None:
        self.filter.shard_insert_hi_dev(local32.data_ptr(), local32.numel(), hi, stream=self._stream())

    def shard_test_hi(self, local32: torch.Tensor, hi: int, out: torch.Tensor) -> None:
        self.filter.shard_test_hi_dev(local32.data_ptr(), local32.numel(), hi, out.data_ptr(), stream=self._stream())

    def shard_insert(self, local: torch.Tensor) -> None:
        self.filter.shard_insert_dev(local.data_ptr(), local.numel(), stream=self._stream())

    def shard_test(self, local: torch.Tensor) -> torch.Tensor:
        out = torch.empty(local.numel(), dtype=torch.uint8, device=self.device)
        self.filter.shard_test_dev(local.data_ptr(), local.numel(), out.data_ptr(), stream=self._stream())
        return out

    def combine(self, bits: torch.Tensor, slot: torch.Tensor, n: int) -> torch.Tensor:
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self.filter.combine_dev(bits.data_ptr(), slot.data_ptr(), n, out.data_ptr(), stream=self._stream())
        return out

    def clear(self) -> None:
        self.filter.clear() if self.P == 1 else self.filter.shard_import(b"")

    def shard_export(self) -> np.ndarray:
        torch.cuda.current_stream(self.device).synchronize()
        return self.filter.shard_export()

    def shard_tensor(self) -> torch.Tensor:
        """The shard's local bytes as a device tensor VIEW of the bitset (no copy): what the
        export gather sends over RCCL."""
        return device_bytes_view(self.filter, (self.filter.local_bits + 7) // 8)

    def shard_import(self, local: np.ndarray) -> None:
        torch.cuda.current_stream(self.device).synchronize()
        self.filter.shard_import(local[: (self.filter.local_bits + 7) // 8].tobytes())

    def close(self):
        self.filter.close()


class _DevBytes:
    """Raw device bytes exposed to torch through __cuda_array_interface__."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def device_bytes_view(f: Filter, nbytes: Optional[int] = None) -> torch.Tensor:
    """A uint8 torch tensor aliasing a filter's device bitset (Redis byte order)."""
    ptr, total = f.device_bits()
    dev = torch.device("cuda", f.device if f.device >= 0 else torch.cuda.current_device())
    return torch.as_tensor(_DevBytes(ptr, total if nbytes is None else min(nbytes, total)), device=dev)


def or_allreduce_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place bitwise OR of a uint8 tensor over the group.  RCCL has no bitwise-OR
    reduction (ncclRedOp_t: sum / prod / max / min / avg), so it is built as SURVEY §8(e)
    (ii) says: all_to_all (rank r receives every rank's r-th chunk) -> local OR ->
    all_gather of the OR-ed chunks; each rank moves 2 (P-1)/P of the tensor, like a ring
    all-reduce."""
    P = dist.get_world_size(group)
    if P == 1 or t.numel() == 0:
        return t
    n = t.numel()
    per = -(-n // (P * 16)) * 16                  # chunks of whole 16-B vectors
    buf = torch.zeros(P * per, dtype=torch.uint8, device=t.device)
    buf[:n] = t
    recv = torch.empty_like(buf)
    _all_to_all_single(recv, buf, group=group)
    parts = recv.view(P, per // 8, 8).view(torch.int64).view(P, per // 8)
    acc = parts[0].clone()
    for r in range(1, P):
        acc.bitwise_or_(parts[r])
    _all_gather_into_tensor(buf, acc.view(torch.uint8).view(-1), group=group)
    t.copy_(buf[:n])
    return t


def _device_batch(keys, device) -> Tuple[torch.Tensor, torch.Tensor, int]:
    buf, offs = _keys.pack(keys)
    kb = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(device)
    ko = torch.from_numpy(offs.view(np.int64)).to(device)
    return kb, ko, len(offs) - 1


def _prefix(counts) -> List[int]:
    return np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64).tolist() if len(counts) else []


class PartitionedFilter:
    """A filter block-cyclically partitioned over the ranks of a process group.

    windows=True (default): the route writes each owner's probes straight into a fixed
    window of the send buffer (bf_route_windows_dev) and the windows go out as one group of
    sends/receives, so no pass regroups them owner-major; a batch that overflows a window
    takes the contiguous bf_route_dev path instead (same exchange, same answers)."""

    WINDOW_ALIGN = 12288   # BF_WINDOW_CAP_ALIGN: windows the owner's binned path can take whole

    def __init__(self, m: int, k: int, block_log2: int = 20, group=None, device=None, engine=None,
                 windows: bool = True, pack_answers: bool = True, sync_free: bool = True,
                 batch_capacity: Optional[int] = None, poison: Optional[int] = None, chunks: bool = True,
                 hash_split: bool = True):
        self.group = group
        self.P = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.m, self.k, self.block_log2 = int(m), int(k), int(block_log2)
        self.reach_bits = min(self.m, self.k * 0xFFFFFFFF + 1)
        if engine is None:
            device = device or torch.device("cuda", torch.cuda.current_device())
            engine = HipEngine(self.m, self.k, self.P, self.rank, self.block_log2, device)
        self.engine = engine
        self.device = engine.device
        self.windows = windows
        self.pack_answers = pack_answers   # window route: include? answers return as bits
        self.window_overflows = 0
        # sync-free exchange: whole windows travel, counts stay on the device (needs the
        # window route and the engine's windowed owner ops)
        self.sync_free = bool(sync_free and windows and hasattr(engine, "shard_insert_windows"))
        self.replays = 0
        self._pk_seg = {}
        self._pending = None
        # next_include (insert_include_dev): the SHA-1 words of the next call's include? batch,
        # hashed by this call's owner test (kb, n, words); that call routes from them
        self._next_inc = None
        self.routed_from_digests = 0   # include? routes that started from next_include's words
        # chunked windows (sync-free exchange on an engine that has them): the route sorts each
        # window's runs by the owner's superbin and sends a directory beside them, so the owner
        # skips its sort pass; BFHIP_CHUNKS=0 keeps the plain windows
        self.chunks = bool(chunks and self.sync_free and hasattr(engine, "route_chunks")
                           and os.environ.get("BFHIP_CHUNKS", "1") != "0")
        # a shard count whose windows have no chunk geometry (P * nh past the directory's
        # window limit, e.g. the k = 13 filters at P = 6) takes the plain sync-free windows;
        # the geometry depends only on the shard layout, so every rank decides the same
        if self.chunks and engine.chunk_info(1) is None:
            self.chunks = False
        self._chunk_geo = {}
        # chunked routes hash in a pass of their own (bf_hash_many_dev, full occupancy), then
        # route from the words (bf_route_chunks_digests_dev): the route's LDS sort holds one
        # workgroup per CU, too few waves to hide SHA-1 behind (200B x 8: 6.61 -> 6.17 ms per
        # rank step, profiles/r06j_sim_P8.jsonl)
        self.hash_split = bool(hash_split and hasattr(engine, "hash_keys"))
        # The sync-free windows are sized from a batch bound every rank agrees on, never from
        # the rank's own n: ranks that size them from different n would post p2p messages of
        # different sizes (undefined under RCCL).  ``batch_capacity`` (the same on every rank)
        # fixes it up front; otherwise the first sync-free call agrees on max n by one
        # all-reduce.  A later call with n past the bound overflows its windows, which every
        # rank sees in the overflow flag, and the synced replay (counts exchanged, any sizes)
        # raises the bound on every rank together.
        self._sf_n = int(batch_capacity) if batch_capacity else None
        self.agreements = 0
        # Test hook: every window buffer of the exchange (send windows, receive windows,
        # returned answers) is filled with a known value before it is written, so that a read
        # of a dead entry is a deterministic wrong bit or answer.  Routed
        # entries get `poison` (an owner-local offset: 1 puts a stray bit where the oracle has
        # none), answer bytes 0 (a stray AND turns a member false).
        if poison is None and os.environ.get("BFHIP_POISON_WINDOWS"):
            poison = int(os.environ["BFHIP_POISON_WINDOWS"], 0)
        self.poison = poison
        if poison is not None and hasattr(engine, "poison"):
            engine.poison = poison

    # -- exchange helpers
    def _splits(self, counts: torch.Tensor):
        """Per-owner send counts -> (send splits, receive splits) on the host (one small
        all-to-all; the host waits for it)."""
        recv_counts = torch.empty_like(counts)
        _all_to_all_single(recv_counts, counts, group=self.group)
        cnt = torch.stack([counts, recv_counts]).cpu()
        return cnt[0].tolist(), cnt[1].tolist()

    def _cap(self, n: int) -> int:
        """Window size for a batch of n keys: the block-cyclic map spreads probes evenly, so
        1/P of them plus 12.5 % and a small-batch slack (a sub-range window of a split owner
        gets the owner's whole share); a skewed batch (e.g. one key repeated) overflows and
        is routed again with cap = n*k."""
        probes = n * self.k
        return min(probes, probes // self.P + probes // (8 * self.P) + 4096)

    def _route_start(self, kb, ko, n: int, want_slot: bool) -> dict:
        """Enqueue a batch's route and the all-to-all of its counts; nothing waits here, so
        the next batch's route can be enqueued before the host needs these counts."""
        e = self.engine
        if self.windows and hasattr(e, "route_windows"):
            cap = self._cap(n)
            send, slot, counts = e.route_windows(kb, ko, n, cap, want_slot=want_slot)
        else:
            cap = None
            send, slot, counts = e.route(kb, ko, n, want_slot=want_slot)
        recv_counts = torch.empty_like(counts)
        work = _all_to_all_single(recv_counts, counts, group=self.group, async_op=True)
        return dict(kb=kb, ko=ko, n=n, want_slot=want_slot, send=send, slot=slot, counts=counts,
                    recv_counts=recv_counts, work=work, cap=cap)

    def _route_finish(self, st: dict) -> dict:
        """Wait for the counts (host) and build the exchange: the send buffer, slots, device
        counts and the segment lists ``sseg`` = [(peer, offset, count)] to send and ``rseg`` =
        [(peer, offset, count)] to receive, in the order the two sides agree on, plus ``hruns``
        = [(hi, start, end)] of the receive buffer for the owner ops (window route: one run
        per 2^32-bit sub-range)."""
        e, P, n, want_slot = self.engine, self.P, st["n"], st["want_slot"]
        st["work"].wait()
        cnt = torch.stack([st["counts"], st["recv_counts"]]).cpu()
        sc, rc = cnt[0].tolist(), cnt[1].tolist()
        send, slot, counts, cap = st["send"], st["slot"], st["counts"], st["cap"]
        if cap is not None:
            nh = e.nh
            if max(sc) > cap:
                # A window past cap holds undefined entries: route again into windows that
                # always fit.  Each rank decides alone and the counts are the same, so the
                # exchange below does not change shape.
                self.window_overflows += 1
                cap = max(n * self.k, 1)
                send, slot, counts = e.route_windows(st["kb"], st["ko"], n, cap, want_slot=want_slot)
            sseg = [(o, (o * nh + h) * cap, sc[o * nh + h]) for o in range(P) for h in range(nh)]
            rseg, hruns, at = [None] * (P * nh), [], 0
            for h in range(nh):   # receive buffer: sub-range major, then source
                h0 = at
                for src in range(P):
                    rseg[src * nh + h] = (src, at, rc[src * nh + h])
                    at += rc[src * nh + h]
                hruns.append((h, h0, at))
            rt = dict(send=send, slot=slot, counts=counts, cap=cap, sseg=sseg, rseg=rseg, hruns=hruns, total=at)
            if want_slot and self.pack_answers and hasattr(e, "pack_answers"):
                # the answers return as bits: segment (src, h) packs to ceil(count / 8) bytes,
                # window w lands at w * ceil(cap / 8) on the requester
                cap8 = (cap + 7) // 8
                pk = [(c + 7) // 8 for _, _, c in rseg]
                pd = _prefix(pk)
                rt["pseg"] = torch.tensor([[off, c, d] for (_, off, c), d in zip(rseg, pd)],
                                          dtype=torch.int64).to(self.device)
                rt["pk_send"] = [(src, d, k_) for (src, _, _), d, k_ in zip(rseg, pd, pk)]
                rt["pk_recv"] = [(o, (off // cap) * cap8, (c + 7) // 8) for o, off, c in sseg]
                rt["pk_total"], rt["pk_max"], rt["cap8"] = sum(pk), max(c for _, _, c in rseg), cap8
            return rt
        sd, rd = _prefix(sc), _prefix(rc)
        return dict(send=send, slot=slot, counts=counts, cap=None,
                    sseg=[(o, sd[o], sc[o]) for o in range(P)], rseg=[(o, rd[o], rc[o]) for o in range(P)],
                    hruns=None, total=sum(rc))

    def _route(self, kb, ko, n: int, want_slot: bool) -> dict:
        return self._route_finish(self._route_start(kb, ko, n, want_slot))

    def _p2p(self, send: torch.Tensor, sseg, recv: torch.Tensor, rseg):
        """Grouped send/recv: each (peer, offset, count) of sseg goes to that peer, each of
        rseg comes from it (an all-to-all whose segments need not be contiguous; one RCCL
        group of ncclSend/ncclRecv on the process group's stream; messages between two
        ranks match in list order).  The self segments are device copies on the current
        stream.  Returns the works to wait on."""
        mine_s = [(o, c) for p_, o, c in sseg if p_ == self.rank]
        mine_r = [(o, c) for p_, o, c in rseg if p_ == self.rank]
        for (so, c), (ro, _) in zip(mine_s, mine_r):
            if c:
                recv[ro: ro + c].copy_(send[so: so + c])

        def g(peer):
            return peer if self.group is None else dist.get_global_rank(self.group, peer)

        sends = [(g(peer), send[off: off + c]) for peer, off, c in sseg if peer != self.rank and c]
        recvs = [(g(peer), recv[off: off + c]) for peer, off, c in rseg if peer != self.rank and c]
        return _batch_p2p(sends, recvs, self.group)

    def _exchange(self, kb, ko, n: int, want_slot: bool):
        """route, then the offsets to their owners (async): returns (recv, route, works)."""
        return self._send_routed(self._route(kb, ko, n, want_slot))

    def _buf(self, n: int, dtype, device, answers: bool = False) -> torch.Tensor:
        """An exchange buffer (uninitialised, or poisoned under the test hook)."""
        t = torch.empty(n, dtype=dtype, device=device)
        if self.poison is not None:
            t.fill_(0 if answers else self.poison)
        return t

    def _send_routed(self, rt: dict):
        recv = self._buf(rt["total"], rt["send"].dtype, rt["send"].device)
        works = self._p2p(rt["send"], rt["sseg"], recv, rt["rseg"])
        return recv, rt, works

    def _shard_insert(self, recv: torch.Tensor, rt: dict) -> None:
        if rt["hruns"] is None:
            self.engine.shard_insert(recv)
            return
        for h, a, b in rt["hruns"]:
            if b > a:
                self.engine.shard_insert_hi(recv[a:b], h)

    def _shard_test(self, recv: torch.Tensor, rt: dict) -> torch.Tensor:
        if rt["hruns"] is None:
            return self.engine.shard_test(recv)
        bits = self._buf(recv.numel(), torch.uint8, recv.device, answers=True)
        for h, a, b in rt["hruns"]:
            if b > a:
                self.engine.shard_test_hi(recv[a:b], h, bits[a:b])
        return bits

    def _answer(self, bits: torch.Tensor, rt: dict, n: int) -> torch.Tensor:
        """Owner answers (one byte per received probe) back to the requesters, then AND per key."""
        cap = rt["cap"]
        if "pseg" in rt:   # one bit per probe on the way back
            packed = self.engine.pack_answers(bits, rt["pseg"], rt["pk_max"], rt["pk_total"])
            back = self._buf(max(rt["counts"].numel() * rt["cap8"], 1), torch.uint8, bits.device, answers=True)
            for w in self._p2p(packed, rt["pk_send"], back, rt["pk_recv"]):
                w.wait()
            return self.engine.combine_windows_packed(back, rt["slot"], rt["counts"], cap, n)
        size = rt["send"].numel() if cap is not None else sum(c for _, _, c in rt["sseg"])
        back = self._buf(size, torch.uint8, bits.device, answers=True)
        for w in self._p2p(bits, rt["rseg"], back, rt["sseg"]):
            w.wait()
        if cap is not None:
            return self.engine.combine_windows(back, rt["slot"], rt["counts"], cap, n)
        return self.engine.combine(back, rt["slot"], n)

    # -- the sync-free exchange: fixed windows, counts on the device --------------------------
    #
    # Every rank sends its whole windows (cap entries each, cap a multiple of WINDOW_ALIGN),
    # so the exchange's shape is known without the counts: the counts travel by an async
    # all_to_all beside it, together with each rank's window-overflow flag, and the owner ops
    # read the live counts on the device.  Nothing on the host waits for the device before
    # the whole batch is enqueued.  The host then waits for one early event (after the routes
    # and the count exchange, long done by then) to learn whether any rank's window
    # overflowed (a skewed batch); only then is the batch replayed through the synced path —
    # inserts are idempotent, and include? answers are recomputed into the same tensor — so
    # the results never depend on it.

    def _cap_sf(self, n: int) -> int:
        a = self.WINDOW_ALIGN
        return -(-self._cap(max(n, 1)) // a) * a

    def _agree_batch(self, n: int) -> None:
        """Collective (every rank calls it at the same point): the window bound becomes the
        largest batch any rank has brought so far."""
        t = torch.tensor([int(n), self._sf_n or 0], dtype=torch.int64, device=self.device)
        _all_reduce(t, dist.ReduceOp.MAX, group=self.group)
        self._sf_n = int(t.max().item())
        self.agreements += 1

    def _chunk_geometry(self):
        """(tiles, dir_bytes) for the agreed batch bound, or None (plain windows)."""
        if not self.chunks:
            return None
        if self._sf_n not in self._chunk_geo:
            self._chunk_geo[self._sf_n] = self.engine.chunk_info(max(self._sf_n, 1))
        return self._chunk_geo[self._sf_n]

    def _sf_start(self, kb, ko, n: int, want_slot: bool, dig=None) -> dict:
        """dig: the batch's SHA-1 words (n x 4 int32), hashed earlier: a chunked route starts
        from them (bf_route_chunks_digests_dev) instead of hashing the keys."""
        e, P, nh = self.engine, self.P, self.engine.nh
        if self._sf_n is None:
            self._agree_batch(n)
        # the same cap on every rank; a batch past the agreed bound overflows (global flag)
        cap = self._cap_sf(self._sf_n)
        geo = self._chunk_geometry()
        if geo is not None and n > self._sf_n:   # past the directory's tiles: overflow the windows instead
            geo = None
        dirb = None
        if geo is not None and dig is not None:
            self.routed_from_digests += 1
            send, slot, counts, dirb = e.route_chunks(dig, None, n, cap, geo[0], geo[1], want_slot=want_slot)
        elif geo is not None and self.hash_split:
            dig = e.hash_keys(kb, ko, n)
            send, slot, counts, dirb = e.route_chunks(dig, None, n, cap, geo[0], geo[1], want_slot=want_slot)
        elif geo is not None:
            send, slot, counts, dirb = e.route_chunks(kb, ko, n, cap, geo[0], geo[1], want_slot=want_slot)
        elif self.chunks:
            # a batch the directories cannot hold: its windows are declared overflowed, so every
            # rank replays the step through the synced path and the bound rises
            send, slot, counts = e.route_windows(kb, ko, n, cap, want_slot=want_slot)
            counts.fill_(cap + 1)
        else:
            send, slot, counts = e.route_windows(kb, ko, n, cap, want_slot=want_slot)
        flag = (counts > cap).any().to(torch.int64).view(1, 1)
        msg = torch.cat([counts.view(P, nh), flag.expand(P, 1)], dim=1).contiguous()
        rmsg = torch.empty_like(msg)   # rmsg[s, h]: source s's count for my window h; [s, nh]: its flag
        work = _all_to_all_single(rmsg, msg, group=self.group, async_op=True)
        sseg = [(o, (o * nh + h) * cap, cap) for o in range(P) for h in range(nh)]
        rseg = [(src, (h * P + src) * cap, cap) for h in range(nh) for src in range(P)]
        recv = self._buf(nh * P * cap, send.dtype, send.device)
        works = self._p2p(send, sseg, recv, rseg)
        st = dict(kb=kb, ko=ko, n=n, cap=cap, send=send, slot=slot, counts=counts, rmsg=rmsg, work=work,
                  recv=recv, works=works, geo=None, own_chunks=dirb is not None)
        if self.chunks:
            # every rank sends directories when chunked windows are on: a rank whose batch took
            # plain windows (declared overflowed) still posts them, so the message sizes match
            tiles, dbytes = self._chunk_geometry() or (0, 0)
            if dbytes:
                if dirb is None:
                    dirb = torch.zeros(P * nh * dbytes, dtype=torch.uint8, device=send.device)
                dseg = [(o, (o * nh + h) * dbytes, dbytes) for o in range(P) for h in range(nh)]
                drseg = [(src, (h * P + src) * dbytes, dbytes) for h in range(nh) for src in range(P)]
                rdir = torch.empty(nh * P * dbytes, dtype=torch.uint8, device=send.device)
                st["works"] = works + self._p2p(dirb, dseg, rdir, drseg)
                st.update(geo=(tiles, dbytes), dir=dirb, rdir=rdir)
        return st

    def _sf_flag(self, st: dict) -> None:
        """Enqueue the global overflow flag's trip to pinned host memory (after the count
        exchange) and an event behind it."""
        st["work"].wait()
        ovf = st["rmsg"][:, -1].max().view(1)
        host = torch.empty(1, dtype=torch.int64, pin_memory=torch.cuda.is_available() and ovf.is_cuda)
        host.copy_(ovf, non_blocking=True)
        ev = torch.cuda.Event() if ovf.is_cuda else None
        if ev is not None:
            ev.record()
        st["ovf"], st["ovf_ev"] = host, ev

    def _sf_overflowed(self, st: dict) -> bool:
        if st["ovf_ev"] is not None:
            st["ovf_ev"].synchronize()
        return bool(st["ovf"].item())

    def _sf_insert(self, st: dict) -> None:
        e, P, nh, cap = self.engine, self.P, self.engine.nh, st["cap"]
        for w in st["works"]:
            w.wait()
        if st["geo"] is not None:   # every sub-range in one binned pass, no owner sort
            tiles, dbytes = st["geo"]
            e.shard_insert_chunks(st["recv"], cap, P, st["rdir"], dbytes, tiles, st["rmsg"], nh + 1)
            return
        for h in range(nh):
            e.shard_insert_windows(st["recv"][h * P * cap:(h + 1) * P * cap], cap, P, st["rmsg"], h, nh + 1, h)

    def _sf_answer(self, st: dict, next_include=None) -> torch.Tensor:
        """next_include = (kb, ko, n): the owner test also hashes that batch (chunked windows
        only); its words are kept for the call that brings it as its include? batch."""
        e, P, nh, cap, n = self.engine, self.P, self.engine.nh, st["cap"], st["n"]
        for w in st["works"]:
            w.wait()
        side = next_include is not None and next_include[2] and hasattr(e, "hash_keys")
        if st["geo"] is not None and self.pack_answers and not side and hasattr(e, "shard_test_chunks_packed"):
            # the owner test writes the return trip's packed bits itself (no answer bytes, no pack pass)
            tiles, dbytes = st["geo"]
            packed = e.shard_test_chunks_packed(st["recv"], cap, P, st["rdir"], dbytes, tiles, st["rmsg"], nh + 1)
            return self._sf_return_packed(st, packed)
        bits = self._buf(nh * P * cap, torch.uint8, st["recv"].device, answers=True)
        if st["geo"] is not None:
            tiles, dbytes = st["geo"]
            nxt = None
            if next_include is not None and next_include[2] and hasattr(e, "hash_keys"):
                nkb, nko, nn = next_include
                dig = torch.empty((nn, 4), dtype=torch.int32, device=st["recv"].device)
                nxt = (nkb, nko, nn, dig)
                self._next_inc = dict(kb=nkb, ko=nko, n=nn, dig=dig)
            e.shard_test_chunks(st["recv"], cap, P, st["rdir"], dbytes, tiles, st["rmsg"], nh + 1, bits, nxt=nxt)
        else:
            for h in range(nh):
                e.shard_test_windows(st["recv"][h * P * cap:(h + 1) * P * cap], cap, P, st["rmsg"], h, nh + 1, h,
                                     bits[h * P * cap:(h + 1) * P * cap])
        if self.pack_answers and hasattr(e, "pack_answers"):   # one bit per probe on the way back
            cap8 = (cap + 7) // 8
            key = (cap, P, nh)
            if key not in self._pk_seg:   # (src, count, dst): window (src, h) -> packed[(src*nh + h)*cap8]
                self._pk_seg[key] = torch.tensor([[(h * P + src) * cap, cap, (src * nh + h) * cap8]
                                                  for src in range(P) for h in range(nh)],
                                                 dtype=torch.int64).to(bits.device)
            packed = e.pack_answers(bits, self._pk_seg[key], cap, P * nh * cap8)
            back = self._buf(P * nh * cap8, torch.uint8, bits.device, answers=True)
            seg = [(src, (src * nh + h) * cap8, cap8) for src in range(P) for h in range(nh)]
            for w in self._p2p(packed, seg, back, seg):
                w.wait()
            if st["geo"] is not None and not st["own_chunks"]:
                # this rank's batch took plain windows declared overflowed: the step is replayed
                return torch.zeros(n, dtype=torch.uint8, device=bits.device)
            if st["geo"] is not None:
                tiles, dbytes = st["geo"]
                return e.combine_chunks_packed(back, st["slot"], cap, st["dir"], dbytes, tiles, st["counts"], n)
            return e.combine_windows_packed(back, st["slot"], st["counts"], cap, n)
        back = self._buf(P * nh * cap, torch.uint8, bits.device, answers=True)
        sseg = [(src, (h * P + src) * cap, cap) for src in range(P) for h in range(nh)]
        rseg = [(o, (o * nh + h) * cap, cap) for o in range(P) for h in range(nh)]
        for w in self._p2p(bits, sseg, back, rseg):
            w.wait()
        if st["geo"] is not None and not st["own_chunks"]:   # declared overflowed: the step is replayed
            return torch.zeros(n, dtype=torch.uint8, device=bits.device)
        if st["geo"] is not None:   # bytes came back: pack them here for the chunked combine
            tiles, dbytes = st["geo"]
            cap8 = (cap + 7) // 8
            key = ("local", cap, P, nh)
            if key not in self._pk_seg:
                self._pk_seg[key] = torch.tensor([[w * cap, cap, w * cap8] for w in range(P * nh)],
                                                 dtype=torch.int64).to(bits.device)
            packed = e.pack_answers(back, self._pk_seg[key], cap, P * nh * cap8)
            return e.combine_chunks_packed(packed, st["slot"], cap, st["dir"], dbytes, tiles, st["counts"], n)
        return e.combine_windows(back, st["slot"], st["counts"], cap, n)

    def _sf_return_packed(self, st: dict, packed: torch.Tensor) -> torch.Tensor:
        """The owner's packed answers back to their requesters, then this rank's combine."""
        e, P, nh, cap, n = self.engine, self.P, self.engine.nh, st["cap"], st["n"]
        tiles, dbytes = st["geo"]
        cap8 = (cap + 7) // 8
        back = self._buf(P * nh * cap8, torch.uint8, packed.device, answers=True)
        seg = [(src, (src * nh + h) * cap8, cap8) for src in range(P) for h in range(nh)]
        for w in self._p2p(packed, seg, back, seg):
            w.wait()
        if not st["own_chunks"]:   # this rank's batch took plain windows declared overflowed: replayed
            return torch.zeros(n, dtype=torch.uint8, device=packed.device)
        return e.combine_chunks_packed(back, st["slot"], cap, st["dir"], dbytes, tiles, st["counts"], n)

    def _sf_insert_answer(self, st_i: dict, st_q: dict, next_include=None) -> Optional[torch.Tensor]:
        """_sf_insert(st_i) then _sf_answer(st_q) as ONE owner pass over the shard
        (bf_shard_insert_test_chunks_packed_dev), when both batches took chunked windows of the
        same geometry; None when they did not (the caller then makes the two calls).
        next_include = (kb, ko, n): the pass also hashes that batch (kept for the next call)."""
        e = self.engine
        if (st_i["geo"] is None or st_q["geo"] is None or st_i["geo"] != st_q["geo"] or st_i["cap"] != st_q["cap"]
                or not self.pack_answers or not hasattr(e, "shard_insert_test_chunks_packed")):
            return None
        for w in st_i["works"] + st_q["works"]:
            w.wait()
        nxt = None
        if next_include is not None and next_include[2]:
            nkb, nko, nn = next_include
            dig = torch.empty((nn, 4), dtype=torch.int32, device=st_q["recv"].device)
            nxt = (nkb, nko, nn, dig)
            self._next_inc = dict(kb=nkb, ko=nko, n=nn, dig=dig)
        tiles, dbytes = st_q["geo"]
        packed = e.shard_insert_test_chunks_packed(st_i["recv"], st_i["rdir"], st_i["rmsg"], st_q["recv"],
                                                   st_q["rdir"], st_q["rmsg"], st_q["cap"], self.P, dbytes, tiles,
                                                   e.nh + 1, nxt=nxt)
        return self._sf_return_packed(st_q, packed)

    def _synced_insert(self, kb, ko, n: int) -> None:
        recv, rt, works = self._exchange(kb, ko, n, want_slot=False)
        for w in works:
            w.wait()
        self._shard_insert(recv, rt)

    def _synced_include(self, kb, ko, n: int) -> torch.Tensor:
        recv, rt, works = self._exchange(kb, ko, n, want_slot=True)
        for w in works:
            w.wait()
        return self._answer(self._shard_test(recv, rt), rt, n)

    # -- device-resident batch API (keys already in device memory)
    def insert_many_dev(self, kb: torch.Tensor, ko: torch.Tensor, n: int) -> None:
        self._next_inc = None
        if not self.sync_free:
            return self._synced_insert(kb, ko, n)
        st = self._sf_start(kb, ko, n, want_slot=False)
        self._sf_flag(st)
        self._sf_insert(st)
        if self._sf_overflowed(st):   # a skewed or oversized batch: replay it through the synced path
            self.replays += 1
            self._synced_insert(kb, ko, n)
            self._agree_batch(n)

    def include_many_dev(self, kb: torch.Tensor, ko: torch.Tensor, n: int) -> torch.Tensor:
        self._next_inc = None   # next_include words belong to the next insert_include_dev only
        if not self.sync_free:
            return self._synced_include(kb, ko, n)
        st = self._sf_start(kb, ko, n, want_slot=True)
        self._sf_flag(st)
        out = self._sf_answer(st)
        if self._sf_overflowed(st):
            self.replays += 1
            out.copy_(self._synced_include(kb, ko, n))
            self._agree_batch(n)
        return out

    def insert_include_dev(self, ikb: torch.Tensor, iko: torch.Tensor, ni: int,
                           qkb: torch.Tensor, qko: torch.Tensor, nq: int, next_insert=None,
                           next_include=None) -> torch.Tensor:
        """insert_many_dev(ikb, iko, ni) then include_many_dev(qkb, qko, nq), exchanges overlapped.

        ``next_insert`` = (kb, ko, n), sync-free exchange only: the NEXT call's insert batch is
        routed and sent now, so its exchange runs beside this call's owner kernels; the next
        call must then pass that same batch as (ikb, iko, ni).

        ``next_include`` = (kb, ko, n), chunked windows only: this call's owner test also hashes
        the NEXT call's include? batch (dedicated hashing workgroups beside the L2 sweep), and
        that call routes it from the words instead of hashing it in its route.  The next call
        must pass the same batch as (qkb, qko, nq) to use them (any other batch is routed from
        its keys).  Answers are the same either way.  Contract: the batch's key and offset
        tensors must not be refilled in place between the two calls — only their identity is
        checked (the same ``kb`` and ``ko`` objects, the same n), so a ring buffer rewritten
        in place would be routed from stale words.  Any call other than the next
        ``insert_include_dev`` drops the words."""
        # words hashed by the previous call; taken (and dropped) by this call whatever happens
        ni_, self._next_inc = self._next_inc, None
        pend = self._pending
        if pend is not None and not (pend["kb"] is ikb and pend["n"] == ni):
            # Refused without touching the prefetch: completing it here would run collectives
            # (an overflow replay, the bound agreement) on this rank alone while the others go
            # on into their exchanges, and the job would hang.  Every rank must call
            # drain_prefetch() (collective) to complete the prefetched batch.
            raise ArgumentError("insert_include_dev: the insert batch differs from the prefetched next_insert; "
                                "call drain_prefetch() on every rank")
        self._pending = None
        if self.sync_free and self._sf_n is None:
            # the first sync-free call agrees on the bound from every batch it will route, so an
            # include? (or prefetched) batch larger than the insert batch does not overflow
            self._agree_batch(max(ni, nq, next_insert[2] if next_insert is not None else 0))
        if self.sync_free:
            # route(ins) | send(ins) || route(inc) | send(inc) || shard_insert | shard_test |
            # send(back) | combine, all enqueued before the host waits for anything
            st_i = pend if pend is not None else self._sf_start(ikb, iko, ni, want_slot=False)
            dig = (ni_["dig"] if ni_ is not None and ni_["kb"] is qkb and ni_["ko"] is qko and ni_["n"] == nq
                   else None)
            st_q = self._sf_start(qkb, qko, nq, want_slot=True, dig=dig)
            if next_insert is not None:
                self._pending = self._sf_start(*next_insert, want_slot=False)
            self._sf_flag(st_i)
            self._sf_flag(st_q)
            out = self._sf_insert_answer(st_i, st_q, next_include=next_include)
            if out is None:
                self._sf_insert(st_i)
                out = self._sf_answer(st_q, next_include=next_include)
            if self._sf_overflowed(st_i) or self._sf_overflowed(st_q):
                self.replays += 1
                self._synced_insert(ikb, iko, ni)
                out.copy_(self._synced_include(qkb, qko, nq))
                self._agree_batch(max(ni, nq))
            return out
        return self._insert_include_synced(ikb, iko, ni, qkb, qko, nq)

    def drain_prefetch(self) -> None:
        """Complete a prefetched next_insert that no call will consume: its batch is inserted.
        Collective: every rank must call it at the same point (an overflowed prefetch is
        replayed through the synced exchange and the bound agreed again)."""
        pend, self._pending = self._pending, None
        if pend is not None:
            self._sf_flag(pend)
            self._sf_insert(pend)
            if self._sf_overflowed(pend):
                self.replays += 1
                self._synced_insert(pend["kb"], pend["ko"], pend["n"])
                self._agree_batch(pend["n"])

    def _no_pending(self, what: str) -> None:
        """A prefetched next_insert is routed and sent but not yet applied: a call that
        replaces or reads the whole filter would race it or miss it, so it must be consumed
        (insert_include_dev) or completed (drain_prefetch) first."""
        if self._pending is not None:
            raise ArgumentError("%s: a prefetched next_insert is pending; pass it to insert_include_dev "
                                "or call drain_prefetch() first" % what)

    def _insert_include_synced(self, ikb: torch.Tensor, iko: torch.Tensor, ni: int,
                               qkb: torch.Tensor, qko: torch.Tensor, nq: int) -> torch.Tensor:
        """insert_many_dev(ikb, iko, ni) then include_many_dev(qkb, qko, nq), same results,
        with the exchanges overlapped with the other batch's kernels:

            route(ins) | send(ins) || route(inc) | send(inc) || shard_insert | shard_test | send(back) | combine

        The sends/receives run on the process group's own stream, the kernels on the
        current stream; every owner still applies all ranks' inserts before it tests
        (shard_insert precedes shard_test on its stream), so the include? answers see the
        batch's inserts exactly as in the sequential form."""
        # both routes are enqueued before the host waits for the first batch's counts, so the
        # device goes straight on to route(inc) while the host builds send(ins)
        st_i = self._route_start(ikb, iko, ni, want_slot=False)
        st_q = self._route_start(qkb, qko, nq, want_slot=True)
        recv_i, rt_i, w_i = self._send_routed(self._route_finish(st_i))
        recv_q, rt_q, w_q = self._send_routed(self._route_finish(st_q))   # send(inc) overlaps shard_insert
        for w in w_i:
            w.wait()
        self._shard_insert(recv_i, rt_i)                                    # overlaps send(inc)
        for w in w_q:
            w.wait()
        return self._answer(self._shard_test(recv_q, rt_q), rt_q, nq)

    # -- host API (each rank passes its own keys)
    def insert_many(self, keys: Iterable) -> None:
        kb, ko, n = _device_batch(keys, self.device)
        self.insert_many_dev(kb, ko, n)

    def include_many(self, keys: Iterable) -> np.ndarray:
        kb, ko, n = _device_batch(keys, self.device)
        return self.include_many_dev(kb, ko, n).cpu().numpy().astype(bool)

    def insert_include(self, insert_keys: Iterable, probe_keys: Iterable) -> np.ndarray:
        """insert_many(insert_keys) then include_many(probe_keys), exchanges overlapped."""
        ikb, iko, ni = _device_batch(insert_keys, self.device)
        qkb, qko, nq = _device_batch(probe_keys, self.device)
        return self.insert_include_dev(ikb, iko, ni, qkb, qko, nq).cpu().numpy().astype(bool)

    def clear(self) -> None:
        self._no_pending("clear")
        self.engine.clear()

    # -- Redis string (collective: every rank must call)
    def _shard_tensor(self) -> torch.Tensor:
        if hasattr(self.engine, "shard_tensor"):
            return self.engine.shard_tensor()
        return torch.from_numpy(self.engine.shard_export())

    def export_redis(self, dst: int = 0) -> Optional[bytes]:
        """The trimmed Redis string, assembled on rank ``dst`` (None on the others).  The
        shards travel one at a time into one preallocated buffer of the largest shard's size
        (device memory under RCCL), so no rank but ``dst`` ever holds more than its own shard
        and ``dst`` holds the string once, on the host."""
        self._no_pending("export_redis")
        mine = self._shard_tensor()
        bb = (1 << self.block_log2) // 8
        nblocks = (self.reach_bits + (1 << self.block_log2) - 1) >> self.block_log2
        if self.rank != dst:
            if mine.numel():
                _send(mine, dist.get_global_rank(self.group, dst) if self.group is not None else dst,
                      group=self.group)
            return None
        out = np.zeros(nblocks * bb, dtype=np.uint8)
        view = out.reshape(nblocks, bb)
        big = (shard_local_bits(self.reach_bits, self.P, 0, self.block_log2) + 7) // 8
        buf = torch.empty(big, dtype=torch.uint8, device=mine.device)
        for s_ in range(self.P):
            cnt = len(range(s_, nblocks, self.P))
            if cnt == 0:
                continue
            nb = (shard_local_bits(self.reach_bits, self.P, s_, self.block_log2) + 7) // 8
            if s_ == self.rank:
                part = mine[:nb]
            else:
                _recv(buf[:nb], dist.get_global_rank(self.group, s_) if self.group is not None else s_,
                      group=self.group)
                part = buf[:nb]
            host = part.cpu().numpy()
            if len(host) < cnt * bb:   # a whole-filter handle (P == 1) stops at the reachable prefix
                host = np.concatenate([host, np.zeros(cnt * bb - len(host), np.uint8)])
            view[s_::self.P] = host[: cnt * bb].reshape(cnt, bb)
        out = out[: (self.reach_bits + 7) // 8]
        nz = np.flatnonzero(out)
        return out[: nz[-1] + 1].tobytes() if len(nz) else b""

    def write_redis(self, redis, key: str, chunk_bytes: int = 8 << 20, replace: bool = True) -> int:
        """Write the filter to ``key`` with every rank sending its own blocks (SETRANGE at the
        block's place in the string), so nothing is gathered anywhere.  Collective.  The
        string's length is the global last nonzero byte + 1 (one all-reduce): every write is
        clipped to it, all-zero blocks are skipped, and the block holding that last byte
        grows the key to exactly the length the SETBITs would have.
        ``replace``: rank 0 DELs the key first (a barrier orders it before the writes).
        Returns the bytes this rank sent."""
        self._no_pending("write_redis")
        local = self.engine.shard_export()
        bb = (1 << self.block_log2) // 8
        nz = np.flatnonzero(local)
        last = -1
        if len(nz):   # the local byte -> its place in the string
            lb = int(nz[-1])
            last = ((lb // bb) * self.P + self.rank) * bb + lb % bb
        t = torch.tensor([last], dtype=torch.int64, device=self._shard_tensor().device)
        _all_reduce(t, dist.ReduceOp.MAX, group=self.group)
        length = int(t.item()) + 1
        if replace and self.rank == 0:
            redis.delete(key)
        dist.barrier(group=self.group)
        sent = 0
        for j in range(len(local) // bb + (1 if len(local) % bb else 0)):
            off = (j * self.P + self.rank) * bb
            if off >= length:
                break
            blk = local[j * bb: (j + 1) * bb][: length - off]
            if not blk.any():
                continue
            for c in range(0, len(blk), chunk_bytes):
                part = blk[c: c + chunk_bytes]
                redis.setrange(key, off + c, part.tobytes())
                sent += len(part)
        dist.barrier(group=self.group)
        return sent

    def import_redis(self, data: bytes) -> None:
        self._no_pending("import_redis")
        self.engine.shard_import(split_shard(data, self.P, self.rank, self.reach_bits, self.block_log2))

    def close(self):
        self.engine.close()


def merge_gathered(gk: torch.Tensor, gl: torch.Tensor, sizes, max_b: int, max_n: int, skip: int):
    """The all-gathered batches (rank r's key bytes at gk[r*max_b ..], its key lengths at
    gl[r*max_n ..]; sizes[r] = (bytes, keys, max length)) except rank `skip`'s, as ONE packed
    batch: (key bytes + 16 B slack, int64 offsets[n+1], n)."""
    parts_b, parts_l = [], []
    for r, (nb, cnt, _) in enumerate(sizes):
        if r == skip or cnt == 0:
            continue
        parts_b.append(gk[r * max_b: r * max_b + nb])
        parts_l.append(gl[r * max_n: r * max_n + cnt])
    n = sum(int(x.numel()) for x in parts_l)
    if n == 0:
        return None, None, 0
    kb = torch.cat(parts_b + [torch.zeros(16, dtype=torch.uint8, device=gk.device)])
    offs = torch.zeros(n + 1, dtype=torch.int64, device=gk.device)
    torch.cumsum(torch.cat(parts_l).to(torch.int64), 0, out=offs[1:])
    return kb, offs, n


class ReplicatedFilter:
    """Every rank holds the whole filter; include? is local.  An insert reaches every replica
    one of two ways (SURVEY §8 e):

    * ``"gather"`` (i): the key batches are all-gathered and every replica inserts all of
      them — about L + 1 bytes per key on the wire, but the insert work grows with P;
    * ``"or"`` (ii): every replica inserts only its own batch, then the bitsets are
      OR-all-reduced (``or_allreduce_``) — 2 (P-1)/P of the bitset on the wire per rank,
      the insert work stays flat;
    * ``"digests"``: (i) with every key hashed once, by its own rank: the 16-B SHA-1 words
      (``ruby.rb:42-47``'s h[0..3]) are all-gathered and every replica inserts all of them
      from words (no hash pass) — 16 B per key on the wire instead of ~L + 1, and P - 1
      fewer SHA-1 passes per replica (``tools/sim_rank.py --replicated P --gathered``);
    * ``"sets"``: (i) with every batch also SORTED once, by its own rank: each rank encodes its
      batch as per-region Elias-Fano sets of the offsets it probes
      (``bf_encode_region_sets_dev``, about the SHA-1 words' size on the wire), the fixed-size
      set buffers are all-gathered, and every replica ORs all of them in with one pass over
      its bitset and no sort (``bf_insert_region_sets_dev``): a replica's insert work no
      longer repeats every other rank's sort.

    ``insert_mode="auto"`` takes (ii) when the bitset is small next to the gathered batches
    (2 * bitset bytes < all ranks' key bytes + lengths), e.g. the 1M@1 % filter (1.2 MB)
    against 2^24-key batches, and (i) otherwise, e.g. the north-star filter (1.2 GB)."""

    MODES = ("auto", "gather", "or", "digests", "sets")

    def __init__(self, m: int, k: int, group=None, device=None, insert_mode: str = "auto",
                 side_encode: bool = True):
        """side_encode ("sets" mode): a batch given as SHA-1 words (the pipelined step) is encoded
        by a second, bitset-less handle (BF_FLAG_ENCODER) on a stream of its own, so it runs
        beside this replica's apply of the previous batch instead of after it (one handle orders
        all of its calls)."""
        if insert_mode not in self.MODES:
            raise ArgumentError("insert_mode must be one of %s" % (self.MODES,))
        self.group = group
        self.P = dist.get_world_size(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.filter = Filter(m, k, device=self.device.index)
        self.k = k
        self.insert_mode = insert_mode
        self.last_insert_mode = None
        self.host_wait_s = 0.0   # time the host spent waiting for batch sizes (gather_start)
        # "sets": the apply ORs a device status word when it skips a buffer or a region (a header
        # that does not match, an entry past its buffer, an encode past its capacity).  Its value
        # after each apply is copied to pinned memory behind an event; _sets_check reads the copy
        # two inserts later (by then the pipelined caller's host has already waited past that
        # apply), so no step waits for its own apply.  Every replica applies the same gathered
        # buffers, so every rank sees the same value at the same call and raises together.
        self._sets_status = None
        self._sets_host = None
        self._sets_pending = []   # (insert number, event, pinned slot)
        self._sets_done = 0
        if insert_mode == "sets":
            # a filter that cannot take region sets at all (a non-ruby engine, regions with no
            # set geometry) is refused here; the per-batch fallback to the digests form in
            # gather_start is only for a batch too large for one encode pass
            try:
                self.filter.region_sets_capacity(1)
            except (ArgumentError, BfHipError) as e:
                self.filter.close()
                raise ArgumentError("insert_mode='sets': this filter cannot take region sets (%s)" % e)
        self.encoder = self.enc_stream = None
        if insert_mode == "sets" and side_encode and self.device.type == "cuda":
            self.encoder = Filter(m, k, device=self.device.index, flags=BF_FLAG_ENCODER)
            self.enc_stream = torch.cuda.Stream(self.device)

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def insert_many_dev(self, kb: torch.Tensor, ko: torch.Tensor, n: int) -> None:
        """Every rank's batch reaches every replica; OR is order-free, so the replicas end
        byte-identical to one filter that took the batches in any order.

        gather: the key bytes and one length per key (uint8 while every key fits 255 bytes,
        else int32) are all-gathered while this rank's own batch is inserted, then the
        other ranks' batches go in as ONE insert (one binned pass over the bitset).
        or: this rank's batch, then the bitset OR-all-reduced."""
        st = self.gather_start(kb, ko, n)
        if st["mode"] == "gather" and n:   # own batch, beside the gather
            self.filter.insert_many_dev(kb.data_ptr(), ko.data_ptr(), n, stream=self._stream())
            self.insert_gathered(st, own_inserted=True)
        else:
            self.insert_gathered(st)

    def sizes_start(self, kb: torch.Tensor, ko: torch.Tensor, n: int) -> dict:
        """Enqueue the all-gather of this batch's sizes (collective) and their copy to pinned
        host memory behind an event; ``gather_start(..., sizes=)`` then reads them without
        draining the device.  A caller that starts the sizes one batch ahead of the gather (the
        bench's pipelined step) never makes the host wait for in-flight kernels."""
        z = torch.zeros(1, dtype=torch.int64, device=self.device)
        # the key lengths (and the longest) only for the forms that gather key bytes: the region
        # sets and SHA-1 word forms never read them, and at 2^24 keys they are a 134 MB pass
        # plus a reduction on every step
        need_lens = n and self.insert_mode not in ("sets", "digests")
        lens = (ko[1: n + 1] - ko[:n]) if need_lens else z[:0]
        # (bytes, keys, longest key (0 when not needed), first offset)
        sizes = torch.cat([ko[n: n + 1] - ko[0:1], z + n, lens.max().view(1) if need_lens else z, ko[0:1]])
        all_sizes = torch.empty(self.P * 4, dtype=torch.int64, device=self.device)
        _all_gather_into_tensor(all_sizes, sizes, group=self.group)
        dev = all_sizes.is_cuda
        host = torch.empty(self.P * 4, dtype=torch.int64, pin_memory=dev)
        host.copy_(all_sizes, non_blocking=dev)
        ev = None
        if dev:
            ev = torch.cuda.Event()
            ev.record()
        return dict(host=host, ev=ev, lens=lens, n=n)

    def gather_start(self, kb: torch.Tensor, ko: torch.Tensor, n: int, sizes: Optional[dict] = None,
                     digests: Optional[torch.Tensor] = None) -> dict:
        """Enqueue the all-gather of this rank's batch (collective: every rank calls it, in
        the same order); ``insert_gathered`` finishes it.  Between the two the gather runs on
        the process group's stream beside whatever the caller enqueues — e.g. the previous
        batch's inserts and include?s, so a pipelined caller hides the exchange.  The batch
        sizes come from ``sizes`` (a ``sizes_start`` of this batch issued earlier: the host
        waits only for that small all-gather's event) or from a sizes_start made here (the
        host then waits for everything enqueued before it).  In "or" mode nothing travels
        here; ``insert_gathered`` inserts and OR-all-reduces.  ``digests`` ("sets" mode): the
        batch's SHA-1 words, already computed (e.g. by a fused include?+hash kernel), so the
        encode skips its hash pass."""
        if sizes is None:
            sizes = self.sizes_start(kb, ko, n)
        if sizes["n"] != n:
            raise ArgumentError("gather_start: sizes were taken for a batch of %d keys, not %d" % (sizes["n"], n))
        if sizes["ev"] is not None:
            t0 = time.perf_counter()
            sizes["ev"].synchronize()
            self.host_wait_s += time.perf_counter() - t0
        lens = sizes["lens"]
        all_sizes = sizes["host"].view(self.P, 4).tolist()
        nbytes, _, _, ko0 = all_sizes[dist.get_rank(self.group)]
        all_sizes = [sz[:3] for sz in all_sizes]
        mode = self.insert_mode
        if mode == "auto":
            wide = max(sz[2] for sz in all_sizes) > 255
            gather_bytes = sum(sz[0] + sz[1] * (4 if wide else 1) for sz in all_sizes)
            mode = "or" if 2 * self.filter.device_bytes < gather_bytes else "gather"
        if mode == "or":
            return dict(mode="or", kb=kb, ko=ko, n=n)
        if mode == "sets":
            # every rank sizes the buffers from the largest batch of all ranks, so a batch one
            # encode cannot take (more than one binned pass) is found on every rank at once, and
            # they all take the digests form for it together (an error on one rank alone would
            # leave the others waiting in the all-gather)
            try:
                cap = self.filter.region_sets_capacity(max(max(sz[1] for sz in all_sizes), 1))
            except ArgumentError:
                mode = "digests"
        if mode == "sets":   # this rank sorts and encodes its batch once; the region sets travel
            if digests is not None and n and self.encoder is not None:
                # on the encoder's stream, beside whatever this replica's handle runs next (the
                # previous batch's apply); it waits only for what is enqueued so far (the words)
                side = self.enc_stream
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    mine = torch.empty(cap // 4, dtype=torch.int32, device=self.device)
                    self.encoder.encode_region_sets_digests_dev(digests.data_ptr(), n, mine.data_ptr(), cap,
                                                                stream=side.cuda_stream)
                    gs = torch.empty(self.P * (cap // 4), dtype=torch.int32, device=self.device)
                    works = [_all_gather_into_tensor(gs, mine, group=self.group, async_op=True)]
                    ev = torch.cuda.Event()
                    ev.record(side)
                digests.record_stream(side)
                return dict(mode="sets", kb=kb, ko=ko, n=n, gs=gs, send=mine, works=works, sizes=all_sizes, cap=cap,
                            ev=ev)
            mine = torch.empty(cap // 4, dtype=torch.int32, device=self.device)
            if digests is not None and n:
                self.filter.encode_region_sets_digests_dev(digests.data_ptr(), n, mine.data_ptr(), cap,
                                                           stream=self._stream())
            else:
                self.filter.encode_region_sets_dev(kb.data_ptr() if n else 0, ko.data_ptr() if n else 0, n,
                                                   mine.data_ptr(), cap, stream=self._stream())
            gs = torch.empty(self.P * (cap // 4), dtype=torch.int32, device=self.device)
            works = [_all_gather_into_tensor(gs, mine, group=self.group, async_op=True)]
            return dict(mode="sets", kb=kb, ko=ko, n=n, gs=gs, send=mine, works=works, sizes=all_sizes, cap=cap)
        if mode == "digests":   # this rank hashes its batch once; the words travel
            max_n = max(max(sz[1] for sz in all_sizes), 1)
            mine = torch.zeros((max_n, 4), dtype=torch.int32, device=self.device)
            if n and digests is not None:   # already hashed (a pipelined caller)
                mine[:n].copy_(digests[:n])
            elif n:
                self.filter.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n, mine.data_ptr(), stream=self._stream())
            gd = torch.empty((self.P * max_n, 4), dtype=torch.int32, device=self.device)
            works = [_all_gather_into_tensor(gd.view(-1), mine.view(-1), group=self.group, async_op=True)]
            return dict(mode="digests", kb=kb, ko=ko, n=n, gd=gd, send=mine, works=works, sizes=all_sizes,
                        max_n=max_n)
        max_b = max(max(sz[0] for sz in all_sizes), 1)
        max_n = max(max(sz[1] for sz in all_sizes), 1)
        ldt = torch.uint8 if max(sz[2] for sz in all_sizes) <= 255 else torch.int32
        kb_p = torch.zeros(max_b, dtype=torch.uint8, device=self.device)
        if nbytes:
            kb_p[:nbytes] = kb[ko0: ko0 + nbytes]
        ln_p = torch.zeros(max_n, dtype=ldt, device=self.device)
        ln_p[:n] = lens.to(ldt)
        gk = torch.empty(self.P * max_b, dtype=torch.uint8, device=self.device)
        gl = torch.empty(self.P * max_n, dtype=ldt, device=self.device)
        works = [_all_gather_into_tensor(gk, kb_p, group=self.group, async_op=True),
                 _all_gather_into_tensor(gl, ln_p, group=self.group, async_op=True)]
        return dict(mode="gather", kb=kb, ko=ko, n=n, gk=gk, gl=gl, send=(kb_p, ln_p), works=works,
                    sizes=all_sizes, max_b=max_b, max_n=max_n)

    def insert_gathered(self, st: dict, own_inserted: bool = False) -> None:
        """Finish ``gather_start``: every rank's batch goes in — this rank's own with the
        others as ONE insert (one binned pass over the bitset) unless ``own_inserted``."""
        self.last_insert_mode = st["mode"]
        if st["mode"] == "or":
            if st["n"]:
                self.filter.insert_many_dev(st["kb"].data_ptr(), st["ko"].data_ptr(), st["n"], stream=self._stream())
            or_allreduce_(device_bytes_view(self.filter), self.group)
            return
        for w in st["works"]:
            w.wait()
        if st.get("ev") is not None:   # encoded on the encoder's stream (a host-staged gather copies there too)
            torch.cuda.current_stream(self.device).wait_event(st["ev"])
            st["gs"].record_stream(torch.cuda.current_stream(self.device))
        if st["mode"] == "sets":   # every rank's sets ORed in by one pass over the bitset
            probes = sum(sz[1] for sz in st["sizes"]) * self.k
            if probes:
                if self._sets_status is None:
                    self._sets_status = torch.zeros(1, dtype=torch.int32, device=self.device)
                    self._sets_host = torch.zeros(3, dtype=torch.int32, pin_memory=self._sets_status.is_cuda)
                # each apply ORs into a fresh word, so each pinned slot holds that insert's own status
                self._sets_status.zero_()
                self.filter.insert_region_sets_dev(st["gs"].data_ptr(), st["cap"], self.P, probes,
                                                   d_status=self._sets_status.data_ptr(), stream=self._stream())
                self._sets_done += 1
                slot = self._sets_done % 3
                self._sets_host[slot:slot + 1].copy_(self._sets_status, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                self._sets_pending.append((self._sets_done, ev, slot))
                self._sets_check(lag=2)
            return
        if st["mode"] == "digests":   # every rank's words as ONE insert (padding rows cut out)
            counts = [sz[1] for sz in st["sizes"]]
            mx = st["max_n"]
            if all(c == mx for c in counts):
                dg, dn = st["gd"], self.P * mx
            else:
                dg = torch.cat([st["gd"][r * mx: r * mx + c] for r, c in enumerate(counts) if c])
                dn = int(sum(counts))
            if dn:
                self.filter.insert_digests_dev(dg.data_ptr(), dn, stream=self._stream())
            return
        skip = dist.get_rank(self.group) if own_inserted else -1
        ob, oo, on = merge_gathered(st["gk"], st["gl"], st["sizes"], st["max_b"], st["max_n"], skip=skip)
        if on:
            self.filter.insert_many_dev(ob.data_ptr(), oo.data_ptr(), on, stream=self._stream())

    def _sets_check(self, lag: int = 0) -> None:
        """Read the status copies of all but the last ``lag`` region-set inserts; raise if an
        apply skipped a buffer or a region (those inserts are lost: include? would answer
        false for keys that were inserted, the one thing a Bloom filter must never do)."""
        while len(self._sets_pending) > lag:
            no, ev, slot = self._sets_pending.pop(0)
            ev.synchronize()
            if int(self._sets_host[slot]):
                self._sets_pending.clear()
                raise BfHipError(BF_EINVAL, "region-set insert %d: the apply skipped a set buffer or region "
                                            "(foreign, damaged or over-capacity sets); inserts were lost" % no)

    def sets_check(self) -> None:
        """Raise now if any region-set insert so far skipped a buffer or a region (collective
        in effect: every replica applied the same buffers; the host-pointer calls and export do
        this themselves)."""
        self._sets_check(lag=0)

    def include_many_dev(self, kb: torch.Tensor, ko: torch.Tensor, n: int) -> torch.Tensor:
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self.filter.include_many_dev(kb.data_ptr(), ko.data_ptr(), n, out.data_ptr(), stream=self._stream())
        return out

    def insert_many(self, keys: Iterable) -> None:
        kb, ko, n = _device_batch(keys, self.device)
        self.insert_many_dev(kb, ko, n)
        self.sets_check()

    def include_many(self, keys: Iterable) -> np.ndarray:
        kb, ko, n = _device_batch(keys, self.device)
        ans = self.include_many_dev(kb, ko, n).cpu().numpy().astype(bool)
        self.sets_check()
        return ans

    def export_redis(self) -> bytes:
        torch.cuda.current_stream(self.device).synchronize()
        self.sets_check()
        return self.filter.export_redis()

    def close(self):
        if self.encoder is not None:
            self.enc_stream.synchronize()
            self.encoder.close()
        self.filter.close()


class ReplicatedPipeline:
    """The pipelined replicated step (``bench.py --gpus N`` on a replicated layout): a ring of
    batches ``batches[b] = ((insert key bytes, offsets), (include? key bytes, offsets))`` of
    ``n`` keys each, stepped in order (batch b = step number mod len(batches)).  Step i

    1. starts the all-gather of batch i+1 (its sizes were all-gathered during step i-1, so the
       host reads them without waiting for the kernels in flight) and the sizes of batch i+2;
    2. inserts every rank's batch i — this rank's own with the others, as one insert — whose
       gather started during step i-1 (``insert``);
    3. answers include? batch i after those inserts (``include``).

    With ``fused_hash`` ("sets" form): batch i+2's SHA-1 words come out of step i's include?
    kernel (``bf_include_hash_dev``, as the single-GPU step hashes its next batch), so step
    i+1 encodes batch i+2's region sets from words, with no hash pass; the words live in a ring
    of three buffers.  Every key is still hashed once per step.  The answers and every
    replica's bitset equal those of inserting all ranks' batches 0..i before include? i
    (``tests/dist_worker.py``'s ``rpipe`` check).  The last step's gather of the wrapped-around
    batch is left pending: ``drain`` completes it (nothing is inserted from it).

    Errors lag: a region-set apply that skipped a buffer or a region (lost inserts) is raised
    two inserts later (``ReplicatedFilter._sets_check(lag=2)``) so no step waits on its own
    apply; the include? answers of up to two steps can therefore come back before the
    ``BfHipError`` that says they may hold false negatives.  ``drain`` (or
    ``rf.sets_check()``) checks every apply so far."""

    def __init__(self, rf: "ReplicatedFilter", batches, n: int, fused_hash: bool = True):
        self.rf, self.batches, self.n, self.L = rf, batches, n, len(batches)
        if self.L < 1:
            raise ArgumentError("ReplicatedPipeline needs at least one batch")
        # (pending gathers and sizes are keyed by batch index, each taken before it is set again,
        # so any ring length works; the word buffers are keyed by step number)
        self.fused = fused_hash and rf.insert_mode == "sets"
        self.step = 0
        self.gpend, self.szp, self.dig = {}, {}, {}
        if self.fused:   # the pipeline's fill: batches 0 and 1 hashed ahead of step 0
            for b in (0, 1):
                kb, ko = batches[b % self.L][0]
                rf.filter.hash_many_dev(kb.data_ptr(), ko.data_ptr(), n, self._digests(b).data_ptr(),
                                        stream=rf._stream())

    def _digests(self, i: int) -> torch.Tensor:   # step i's batch's SHA-1 words (ring of three)
        if i % 3 not in self.dig:
            self.dig[i % 3] = torch.empty((self.n, 4), dtype=torch.int32, device=self.rf.device)
        return self.dig[i % 3]

    def insert(self) -> None:
        rf, i, L, n = self.rf, self.step, self.L, self.n
        st = self.gpend.pop(i % L, None) or rf.gather_start(*self.batches[i % L][0], n,
                                                              digests=self._digests(i) if self.fused else None)
        nxt = (i + 1) % L
        self.gpend[nxt] = rf.gather_start(*self.batches[nxt][0], n, sizes=self.szp.pop(nxt, None),
                                          digests=self._digests(i + 1) if self.fused else None)
        self.szp[(i + 2) % L] = rf.sizes_start(*self.batches[(i + 2) % L][0], n)
        rf.insert_gathered(st)
        self.step = i + 1

    def include(self, out: torch.Tensor) -> None:
        """include? batch i (the step ``insert`` just finished) into ``out`` (n bytes, 0/1)."""
        rf, i, n = self.rf, self.step - 1, self.n
        pkb, pko = self.batches[i % self.L][1]
        if self.fused:   # ... with batch i+2's SHA-1 fused in
            nkb, nko = self.batches[(i + 2) % self.L][0]
            rf.filter.include_hash_dev(pkb.data_ptr(), pko.data_ptr(), n, out.data_ptr(), nkb.data_ptr(),
                                       nko.data_ptr(), n, self._digests(i + 2).data_ptr(), stream=rf._stream())
        else:
            rf.filter.include_many_dev(pkb.data_ptr(), pko.data_ptr(), n, out.data_ptr(), stream=rf._stream())

    def drain(self) -> None:
        """Complete the pending gathers (collective: every rank calls it after its last step),
        then check every region-set apply so far (raises on every rank alike)."""
        for st in self.gpend.values():
            for w in st.get("works", []):
                w.wait()
        self.gpend.clear()
        if self.rf.insert_mode == "sets":
            self.rf.sets_check()
