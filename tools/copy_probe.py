"""Host copy-rate probe for the storage -> pinned path: 16 threads copying 32 MiB parts of a
4 GiB buffer with a memoryview slice assignment (holds the GIL) vs numpy.copyto (releases it)."""
import concurrent.futures as cf
import time

import numpy as np

n, part = 4 << 30, 32 << 20
src = np.ones(n, np.uint8)
dst = np.zeros(n, np.uint8)
ms, md = memoryview(src), memoryview(dst)


def mv(a):
    md[a:a + part] = ms[a:a + part]


def npc(a):
    np.copyto(dst[a:a + part], src[a:a + part])


for f in (mv, npc, mv, npc):
    t = time.perf_counter()
    with cf.ThreadPoolExecutor(16) as ex:
        list(ex.map(f, range(0, n, part)))
    print(f.__name__, round(n / (time.perf_counter() - t) / 2**30, 2), "GiB/s", flush=True)
