"""Multi-GPU work split: static, no collective on the data path.

An object's FASTA chunk plan is cut into contiguous chunk groups, ``split_groups(nchunks, n_gpus)``, one per
GPU (``scan.objects.fasta_groups``, used by ``co.preprocess`` and by bench.py's threads or ranks); a
newline index's byte range is cut into raw parts (``rank_byte_range``).  Nothing is exchanged between GPUs:
the per-GPU outputs concatenate in order to the whole index.  bench.py's timing barriers / final gather in a
``torch.distributed.run`` launch go over a gloo CPU group; RCCL is never initialised.
"""
from __future__ import annotations

from typing import List, Tuple


def split_groups(n: int, g: int) -> List[Tuple[int, int]]:
    """Contiguous [i0, i1) groups of n items over g workers (the first n % g get one more); no empty
    groups when n < g."""
    g = max(1, min(g, n)) if n > 0 else 1
    q, r = divmod(n, g)
    out, i = [], 0
    for k in range(g):
        j = i + q + (1 if k < r else 0)
        out.append((i, j))
        i = j
    return out


def rank_chunks(nchunks: int, rank: int, world: int) -> Tuple[int, int]:
    """Chunk range of ``rank`` when one object's chunks are spread over ``world`` ranks ([n,n) if none)."""
    groups = split_groups(nchunks, world)
    return groups[rank] if rank < len(groups) else (nchunks, nchunks)


def rank_byte_range(begin: int, end: int, rank: int, world: int) -> Tuple[int, int]:
    """Raw byte range of ``rank`` when one object's [begin, end) is cut into ``world`` parts for a newline
    index (bench.py --workload vcf): ceil-sized parts, so the parts' offset lists concatenate, in rank
    order, to the whole range's index (no boundary adjustment is needed for a delimiter index)."""
    step = -(-(end - begin) // world) if end > begin else 0
    return min(end, begin + rank * step), min(end, begin + (rank + 1) * step)
