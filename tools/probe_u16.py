import sys; sys.path.insert(0, "/root/repo")
import numpy as np
from dataplug_amd import synth
from dataplug_amd.scan import ScanContext
from oracle import dpref
ctx = ScanContext(0)
a = synth.csv((9 << 20) + 17, seed=15)
a[(2 << 20):(2 << 20) + 70_000] = 10
a[(5 << 20):(5 << 20) + 300_000] = ord("x")
d = ctx.workspace("t_in", len(a) + 64)
n = len(a)
for base in (0, 1337):
  ctx.h2d(d.ptr + (base & 15), a)
  for ranges in ([(base, base + n)], [(base, base + 4097), (base + 4097, base + (3 << 20) + 5), (base + (3 << 20) + 5, base + n)]):
    low, nd, ends, tab = ctx.delim_ranges(d.ptr + (base & 15), n, base, ranges, out_mode=3)
    exp = dpref.delim(a, 0, n)[0] + np.uint64(base)
    j0 = base >> 16
    blk = np.searchsorted(tab.astype(np.int64), np.arange(len(low)), side="right").astype(np.uint64) - np.uint64(1)
    got = ((blk + np.uint64(j0)) << np.uint64(16)) | low.astype(np.uint64)
    bounds = np.arange(j0, ((base + n - 1) >> 16) + 1, dtype=np.uint64) << np.uint64(16)
    etab = np.searchsorted(exp, bounds).astype(np.uint64); etab[0] = 0
    badt = np.flatnonzero(tab != etab)
    bad = np.flatnonzero(got != exp)
    lowexp = (exp & np.uint64(0xFFFF)).astype(np.uint16)
    badl = np.flatnonzero(low != lowexp)
    print(base, len(ranges), "nd", nd, len(exp), "bad", len(bad), bad[:5], "badlow", len(badl), badl[:5], "badtab", len(badt), badt[:8], tab[badt[:8]], etab[badt[:8]])
    if len(badl):
        i = badl[0]; print("  low got", low[i-2:i+3], "exp", lowexp[i-2:i+3], "exp off", exp[i-2:i+3])
