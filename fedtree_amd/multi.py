"""Multi-GPU sharding of independent ciphertext batches.

Every ciphertext is independent for encrypt / decrypt / add / scalar-mul, so a
batch splits into contiguous shards, one per GPU, each driven by its own host
thread, engine context (HIP stream) and key copy.  There is no collective on
the data path: inputs and outputs are host-resident (gRPC buffers in FedTree,
distributed_server.cpp:34-53), and the shards never exchange data.  A k-way
product shards by bin range the same way.

Two launch styles use this:
  * in one process (a FedTree server calling encrypt_gh_pairs on 80M pairs):
    ShardedPaillier below, threads x devices;
  * one process per GPU (bench.py under torchrun): shard_range() per rank.
"""
import threading

import numpy as np


def shard_range(total, rank, world):
    """Contiguous [lo, hi) of `total` units owned by `rank` of `world` (balanced to +-1)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class ShardedPaillier:
    """A Paillier key replicated on several devices; batch calls are split
    across them and run concurrently (ctypes releases the GIL in the engine)."""

    def __init__(self, key, devices, bases=None):
        """bases: published fixed-base bases (Paillier.public_bases) for public-key copies'
        encrypt_u64(fixed_base_exact=True); each device builds its own tables."""
        from .paillier import Device, Paillier
        self.devices = [Device(d) if not isinstance(d, Device) else d for d in devices]
        self.keys = []
        for dev in self.devices:
            if key.has_private:
                k = Paillier.from_primes(key.p, key.q, dev)
            else:
                k = Paillier.from_public(key.modulus, dev)
            if bases is not None:
                k.set_public_bases(bases)
            self.keys.append(k)
        self.n_words = key.n_words

    def _run(self, n, fn):
        world = len(self.keys)
        out = [None] * world
        err = [None] * world

        def work(i):
            lo, hi = shard_range(n, i, world)
            try:
                out[i] = fn(self.keys[i], lo, hi)
            except Exception as e:        # re-raised in the caller's thread
                err[i] = e

        ts = [threading.Thread(target=work, args=(i,)) for i in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for e in err:
            if e is not None:
                raise e
        return out

    def encrypt_u64(self, m, seed=0, **modes):
        """modes: public / fixed_base / fixed_base_exact, as Paillier.encrypt_u64."""
        m = np.ascontiguousarray(m, dtype=np.uint64)
        # one stream for the whole batch, each shard at its own positions (index0 = lo): with a nonzero seed the
        # shards give exactly the ciphertexts of one call; seed 0 draws each shard's key from /dev/urandom
        parts = self._run(len(m), lambda k, lo, hi: k.encrypt_u64(m[lo:hi], seed=seed, index0=lo, **modes))
        return np.concatenate(parts) if parts else np.zeros((0, 2 * self.n_words), np.uint32)

    def decrypt_u64(self, c, short=False):
        c = np.ascontiguousarray(c, dtype=np.uint32)
        return np.concatenate(self._run(len(c), lambda k, lo, hi: k.decrypt_u64(c[lo:hi], short=short)))

    def add_batch(self, a, b):
        return np.concatenate(self._run(len(a), lambda k, lo, hi: k.add_batch(a[lo:hi], b[lo:hi])))

    def sub_batch(self, a, b):
        return np.concatenate(self._run(len(a), lambda k, lo, hi: k.sub_batch(a[lo:hi], b[lo:hi])))

    def scalar_mul(self, x, k64):
        return np.concatenate(self._run(len(x), lambda k, lo, hi: k.scalar_mul(x[lo:hi], k64)))

    def reduce_kway(self, x):
        return np.concatenate(self._run(x.shape[1], lambda k, lo, hi: k.reduce_kway(x[:, lo:hi])))

    def sum(self, x):
        """The N-to-1 product of rows x (the root sum of Tree::init_CPU, tree.cpp:20-34, for one plane): each
        device's partial product of its row range (one segment), then the <= 7 partials combined as a k-way
        product on the first device (no collective, a few adds on one side)."""
        x = np.ascontiguousarray(x, dtype=np.uint32)
        parts = self._run(len(x), lambda k, lo, hi: k.reduce_segments(x[lo:hi], np.array([0, hi - lo])))
        stack = np.stack([p[0] for p in parts])                 # (shards, row words)
        if len(stack) == 1:
            return stack[0]
        return self.keys[0].reduce_kway(stack[:, None, :])[0]
