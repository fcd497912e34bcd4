"""Multi-GPU plumbing: one process per GPU, independent objects/chunks, no collective on the data path.

Only the benchmark's bookkeeping crosses ranks (a barrier and two scalar reductions for max-time /
total-bytes), over ``torch.distributed`` (RCCL on the GPU box; ``gloo`` in the CPU tests).  The work split
itself is static: rank r indexes its own object (weak scaling), or, for one object, the contiguous chunk
group ``split_groups(nchunks, world)[r]`` (the same split ``scan.objects`` uses across local GPUs).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple


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


@dataclass
class Dist:
    world: int = 1
    rank: int = 0
    local: int = 0
    backend: Optional[str] = None
    pg: object = None

    @classmethod
    def from_env(cls, backend: str = "nccl") -> "Dist":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        d = cls(world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
        if world > 1:
            import torch
            import torch.distributed as dist
            d.backend = backend
            if backend == "nccl":
                torch.cuda.set_device(d.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", d.local))
            else:
                dist.init_process_group(backend)
            d.pg = dist
        return d

    def _tensor(self, x: float):
        import torch
        dev = f"cuda:{self.local}" if self.backend == "nccl" else "cpu"
        return torch.tensor([float(x)], dtype=torch.float64, device=dev)

    def barrier(self) -> None:
        if self.pg is not None:
            self.pg.barrier()
            if self.backend == "nccl":
                import torch
                torch.cuda.synchronize(self.local)

    def max(self, x: float) -> float:
        if self.pg is None:
            return float(x)
        t = self._tensor(x)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.pg is None:
            return float(x)
        t = self._tensor(x)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

    def close(self) -> None:
        if self.pg is not None:
            self.pg.destroy_process_group()
            self.pg = None
