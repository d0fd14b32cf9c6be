"""Reference (numpy + oracle hashing) implementation of the per-rank engine
primitives of redis-bloomfilter_amd/distributed.py — TEST INFRASTRUCTURE.

Used by the gloo multi-process tests (no GPU) and as the checker for the HIP
engine's route/shard/combine primitives.
"""
import numpy as np
import torch

import pkgload

D = pkgload.load().distributed


class NumpyEngine:
    """Reference implementation of HipEngine's four primitives (CPU, oracle hashing)."""

    def __init__(self, m, k, P, rank, block_log2, orc):
        self.device = torch.device("cpu")
        self.m, self.k, self.P, self.b, self.orc = m, k, P, block_log2, orc
        reach = min(m, k * 0xFFFFFFFF + 1)
        self.local_bits = D.shard_local_bits(reach, P, rank, block_log2)
        self.bits = np.zeros((self.local_bits + 7) // 8, np.uint8)

    def route(self, kb, ko, n, want_slot=True):
        buf = kb.numpy()
        offs = ko.numpy().view(np.uint64)
        idx = self.orc.indexes_many(buf, offs, self.m, self.k).reshape(-1)
        owner, local = D.block_owner_local(idx, self.P, self.b)
        order = np.argsort(owner, kind="stable")
        slot = (np.arange(n * self.k, dtype=np.int64) // self.k)[order].astype(np.int32)   # key of each send entry
        counts = np.bincount(owner, minlength=self.P).astype(np.int64)
        return (torch.from_numpy(local[order].view(np.int64).copy()), torch.from_numpy(slot) if want_slot else None,
                torch.from_numpy(counts))

    def route_windows(self, kb, ko, n, cap, want_slot=True):
        """route() in the window layout; each window's entries shuffled, since the HIP
        route leaves their order unspecified (the exchange must not depend on it)."""
        send, slot, counts = self.route(kb, ko, n, want_slot=True)
        c = counts.numpy()
        wsend = np.zeros(self.P * cap, np.int64)
        wslot = np.full(self.P * cap, -1, np.int32)
        rng = np.random.default_rng(int(c.sum()) + 7)
        at = 0
        for s in range(self.P):
            live = min(int(c[s]), cap)
            perm = at + rng.permutation(int(c[s]))[:live]
            wsend[s * cap: s * cap + live] = send.numpy()[perm]
            wslot[s * cap: s * cap + live] = slot.numpy()[perm]
            at += int(c[s])
        return torch.from_numpy(wsend), torch.from_numpy(wslot) if want_slot else None, counts

    def combine_windows(self, bits, slot, counts, cap, n):
        c = counts.numpy()
        live = np.concatenate([np.arange(s * cap, s * cap + min(int(c[s]), cap)) for s in range(self.P)])
        return self.combine(bits[torch.from_numpy(live)], slot[torch.from_numpy(live)], n)

    def shard_insert(self, local):
        lo = local.numpy().view(np.uint64)
        assert (lo < np.uint64(self.local_bits)).all(), "owner-local offset outside the shard"
        np.bitwise_or.at(self.bits, (lo >> np.uint64(3)).astype(np.int64),
                         (np.uint64(0x80) >> (lo & np.uint64(7))).astype(np.uint8))

    def shard_test(self, local):
        lo = local.numpy().view(np.uint64)
        b = (self.bits[(lo >> np.uint64(3)).astype(np.int64)] >> (np.uint64(7) - (lo & np.uint64(7))).astype(np.uint8)) & 1
        return torch.from_numpy(b.astype(np.uint8))

    def combine(self, bits, slot, n):
        out = np.ones(n, np.uint8)
        out[slot.numpy().astype(np.int64)[bits.numpy() == 0]] = 0
        return torch.from_numpy(out)

    def clear(self):
        self.bits[:] = 0

    def shard_export(self):
        return self.bits.copy()

    def shard_import(self, local):
        self.bits[:] = 0
        self.bits[: len(local)] = local

    def close(self):
        pass
