"""Multi-GPU sharding of a block batch.

FEC blocks are independent (internal/fec/manager.go:119-121: a block is k consecutive source
symbols; encode and recovery touch one block only), so a batch of B blocks is split into
contiguous block ranges, one per rank (one process per GPU), with no collective on the data
path. Only the bench's timing reduction (max over ranks) and optional checksums cross ranks.
"""


def block_range(total_blocks, rank, world):
    """Contiguous [lo, hi) of the global batch owned by `rank`; sizes differ by at most 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total_blocks, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def aggregate_gibps(blocks_per_rank, k, payload_bytes, max_step_seconds):
    """Whole-job payload throughput: every rank's blocks over the slowest rank's step time."""
    total = sum(blocks_per_rank)
    return total * k * payload_bytes / 2**30 / max_step_seconds


def synth_payload_blocks(seed, lo, hi, k, payload_bytes, stride):
    """Deterministic synthetic data shards for global blocks [lo, hi) on the host (numpy):
    byte i of shard j of block b depends only on (seed, b, j, i), so any split of a batch over
    ranks produces the same bytes. Layout [hi-lo, k, stride]: payload, big-endian uint16 length
    trailer (internal/fec/reed_solomon.go:77-87), zero padding."""
    import numpy as np
    nb = hi - lo
    words = (payload_bytes + 7) // 8
    b = np.arange(lo, hi, dtype=np.uint64)[:, None, None]
    j = np.arange(k, dtype=np.uint64)[None, :, None]
    w = np.arange(words, dtype=np.uint64)[None, None, :]
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)) ^ (b << np.uint64(24)) ^ (j << np.uint64(16)) ^ w
        x = x + np.uint64(0x9E3779B97F4A7C15)                      # splitmix64 finaliser
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    out = np.zeros((nb, k, stride), dtype=np.uint8)
    out[:, :, :payload_bytes] = x.view(np.uint8).reshape(nb, k, words * 8)[:, :, :payload_bytes]
    out[:, :, payload_bytes] = (payload_bytes >> 8) & 0xFF
    out[:, :, payload_bytes + 1] = payload_bytes & 0xFF
    return out


_GOLD = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


def _splitmix_fin(x):
    x = (x + _GOLD) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def synth_single_erasures(seed, lo, hi, k):
    """Erased data shard of each global block [lo, hi): splitmix64 of a key no data word uses
    (include/fec_synth.h fec_synth_single_erasures, restated)."""
    import numpy as np
    out = np.empty(hi - lo, dtype=np.int64)
    base = (seed * _GOLD) & _M64
    for i, b in enumerate(range(lo, hi)):
        out[i] = _splitmix_fin(base ^ ((b << 24) & _M64) ^ 0xFFFFFF) % k
    return out
