"""Lane-exact numpy model of scan_kernel<FASTA/DELIM> (dataplug_amd/csrc/dpscan.hip), for CPU validation.

Every wave-level step of the HIP kernel is mirrored on 64-element arrays (one element per lane) with the
same bit formulas, ballots, unit/wave/row geometry, function-form summaries and the 64-lane look-back
window, so logic bugs show up here without a GPU.  Used by tests/test_kernel_model.py.  The model keeps 8 waves per
unit (the kernel now runs 15 data waves + 1 coordinator, and a pipelined schedule); the per-row bit logic,
the function-form summaries and their composition are unchanged by that, and are what this checks.
"""
from __future__ import annotations

import numpy as np

WAVE, WAVES, ROWS = 64, 8, 8
ROW = WAVE * 16
WAVE_BYTES = ROW * ROWS
UNIT = WAVE_BYTES * WAVES
LANES = np.arange(WAVE)
LT = np.array([(1 << l) - 1 for l in range(WAVE)], dtype=object)


def ballot(pred) -> int:
    m = 0
    for l in np.flatnonzero(pred):
        m |= 1 << int(l)
    return m


def clz64(x: int) -> int:
    return 64 - x.bit_length()


def mask16(buf: np.ndarray, pos0: np.ndarray, ch: int) -> np.ndarray:
    b = buf[pos0[:, None] + np.arange(16)[None, :]]
    return ((b == ch) * (1 << np.arange(16))).sum(1).astype(np.int64)


def maybe_has(buf, pos0, ch) -> np.ndarray:
    return (buf[pos0[:, None] + np.arange(16)[None, :]] == ch).any(1)   # exact is a valid "maybe"


def clip16(pos0: np.ndarray, lo: int, hi: int) -> np.ndarray:
    bit = pos0[:, None] + np.arange(16)[None, :]
    return (((bit >= lo) & (bit < hi)) * (1 << np.arange(16))).sum(1).astype(np.int64)


def popc(x: np.ndarray) -> np.ndarray:
    return np.array([bin(int(v)).count("1") for v in x], np.int64)


def fasta_row(buf, pos0, lo, hi, S: int, nxt63: int):
    valid = clip16(pos0, lo, hi)
    gt = mask16(buf, pos0, 62) & valid
    nl = mask16(buf, pos0, 10) & valid
    nb = np.roll(nl & 1, -1)
    nb[63] = nxt63
    V = gt & ~((nl >> 1) | (nb << 15))
    lb = hi - 1 - pos0
    sel = (lb >= 0) & (lb < 16)
    V[sel] &= ~(1 << lb[sel])
    V &= 0xFFFF
    X = V | nl
    R = ((~X) & 0xFFFF) + ((nl << 1) | 1)
    low = nl & (-nl)
    fs = np.where(low != 0, low - 1, 0xFFFF)
    s_last = ((R >> 16) & 1) ^ 1
    H = ballot(nl != 0)
    SB = ballot(s_last != 0)
    S_lane = np.zeros(WAVE, np.int64)
    for l in range(WAVE):
        lt = (1 << l) - 1
        prior = H & lt
        if prior:
            S_lane[l] = int(((SB & lt) >> (63 - clz64(prior))) != 0)
        else:
            S_lane[l] = int(bool(S) or (SB & lt) != 0)
    emits = V & R & np.where(S_lane != 0, ~fs, 0xFFFF) & 0xFFFF
    ends = nl & ((~R) | np.where(S_lane != 0, low, 0)) & 0xFFFF
    s_before = ((S_lane != 0) | ((V & fs) != 0)).astype(np.int64)
    S_out = int(((SB >> (63 - clz64(H))) != 0)) if H else int(bool(S) or SB != 0)
    return V, nl, emits, ends, s_before, H, S_out


def f_then(a, b):
    cF = a[0] + (b[1] if a[2] else b[0])
    sF = b[3] if a[2] else b[2]
    cT = a[1] + (b[1] if a[3] else b[0])
    sT = b[3] if a[3] else b[2]
    return (cF, cT, sF, sT)


IDENT = (0, 0, 0, 1)


def run(buf: np.ndarray, chunks, mode="fasta", delim=10, every_k=1, emit_add=0, pad=16):
    """Returns FASTA (n, 2) pairs or DELIM offsets, computed the way the kernel does (all in one buffer)."""
    size = len(buf)
    b = np.zeros(size + pad + UNIT, np.uint8)
    b[:size] = buf
    chunk_u0, units = [], 0
    for lo, hi in chunks:
        chunk_u0.append(units)
        if hi > lo:
            units += (hi - (lo & ~15) + UNIT - 1) // UNIT
    chunk_u0.append(units)
    desc = [None] * units          # published: ("agg", func) or ("prefix", count, s)
    out = {}
    pending = [-1] * len(chunks)
    total = 0
    for u in range(units):
        c = max(i for i in range(len(chunks)) if chunk_u0[i] <= u)
        lo, hi = chunks[c]
        chunk_first, chunk_last = u == chunk_u0[c], u + 1 == chunk_u0[c + 1]
        ubase = (lo & ~15) + (u - chunk_u0[c]) * UNIT
        wfs, masks = [], []
        for w in range(WAVES):
            wbase = ubase + w * WAVE_BYTES
            if mode == "fasta":
                S = nlseen = fV = 0
                fn_off = -1
                cnt = 0
                mk = []
                for r in range(ROWS):
                    row0 = wbase + r * ROW
                    zero = (np.zeros(WAVE, np.int64), np.zeros(WAVE, np.int64))
                    if row0 >= hi:
                        mk.append(zero)
                        continue
                    pos0 = row0 + LANES * 16
                    need = S or not nlseen or ballot(maybe_has(b, pos0, 62) & (pos0 < hi))
                    if not need:
                        mk.append(zero)
                        continue
                    rend = row0 + ROW
                    nxt = int(b[rend] == 10) if rend < hi else 0
                    V, nl, emits, ends, sb, H, S_out = fasta_row(b, pos0, lo, hi, S, nxt)
                    if not nlseen and H:
                        j0 = (H & -H).bit_length() - 1
                        fV = int(sb[j0])
                        fn_off = r * ROW + j0 * 16 + (int(nl[j0]) & -int(nl[j0])).bit_length() - 1
                        nlseen = 1
                    mk.append((emits.copy(), ends.copy()))
                    cnt += int(popc(emits).sum())
                    S = S_out
                if not nlseen:
                    fV = S
                masks.append((mk, fV, fn_off))
                f = (cnt, cnt - fV, S, S if nlseen else 1)
                if chunk_first and w == 0:
                    f = (f[0], f[0], f[2], f[2])
            else:
                cnt = 0
                mk = []
                for r in range(ROWS):
                    pos0 = wbase + r * ROW + LANES * 16
                    m = mask16(b, pos0, delim) & clip16(pos0, lo, hi)
                    mk.append(m)
                    cnt += int(popc(m).sum())
                masks.append(mk)
                f = (cnt, cnt, 0, 0)
            wfs.append(f)
        unit = wfs[0]
        for f in wfs[1:]:
            unit = f_then(unit, f)
        # look-back with 64-lane windows over the published descriptors
        P, S_in = 0, 0
        if u > 0:
            desc[u] = ("agg", unit)
            acc = IDENT
            j = u - 1
            while True:
                win_desc = [desc[j - l] if j - l >= 0 else ("prefix", 0, 0) for l in range(WAVE)]
                k = next((l for l, d in enumerate(win_desc) if d[0] == "prefix"), WAVE)
                assert all(d is not None for d in win_desc[:k])
                win = IDENT
                for l in range(k - 1, -1, -1):
                    win = f_then(win, win_desc[l][1])
                acc = f_then(win, acc)
                if k < WAVE:
                    pc, ps = win_desc[k][1], win_desc[k][2]
                    P = pc + (acc[1] if ps else acc[0])
                    S_in = acc[3] if ps else acc[2]
                    break
                j -= WAVE
        P_incl = P + (unit[1] if S_in else unit[0])
        S_outu = unit[3] if S_in else unit[2]
        desc[u] = ("prefix", P_incl, S_outu)
        if u + 1 == units:
            total = P_incl
        if mode == "fasta" and chunk_last:
            pending[c] = P_incl - 1 if S_outu else -1
        p, s = P, (0 if chunk_first else S_in)
        wpre = []
        for f in wfs:
            wpre.append((p, s))
            p += f[1] if s else f[0]
            s = f[3] if s else f[2]
        # phase B
        for w in range(WAVES):
            wbase = ubase + w * WAVE_BYTES
            count, S = wpre[w]
            for r in range(ROWS):
                row0 = wbase + r * ROW
                pos0 = row0 + LANES * 16
                if mode == "fasta":
                    mk, fV, fn_off = masks[w]
                    if r == 0:
                        drop = bool(S) and bool(fV)
                        add_end = bool(S) and fn_off >= 0
                    emits, ends = mk[r][0].copy(), mk[r][1].copy()
                    if add_end and fn_off // ROW == r:
                        ends[(fn_off // 16) % 64] |= 1 << (fn_off % 16)
                    if drop:
                        bal = ballot(emits != 0)
                        if bal:
                            l0 = (bal & -bal).bit_length() - 1
                            emits[l0] &= emits[l0] - 1
                            drop = False
                    pc = popc(emits)
                    ex = np.concatenate(([0], np.cumsum(pc)[:-1]))
                    for l in range(WAVE):
                        e = int(emits[l])
                        for bit in range(16):
                            below = bin(e & ((1 << bit) - 1)).count("1")
                            if e >> bit & 1:
                                out[(count + ex[l] + below, 0)] = int(pos0[l]) + bit
                            if int(ends[l]) >> bit & 1:
                                out[(count + ex[l] + below - 1, 1)] = int(pos0[l]) + bit + 1
                    count += int(pc.sum())
                else:
                    m = masks[w][r]
                    pc = popc(m)
                    ex = np.concatenate(([0], np.cumsum(pc)[:-1]))
                    for l in range(WAVE):
                        e = int(m[l])
                        for bit in range(16):
                            if e >> bit & 1:
                                g = count + ex[l] + bin(e & ((1 << bit) - 1)).count("1")
                                if g % every_k == every_k - 1:
                                    out[g // every_k] = int(pos0[l]) + bit + emit_add
                    count += int(pc.sum())
    if mode == "fasta":
        for c, idx in enumerate(pending):       # fasta_resolve_kernel
            if idx >= 0:
                nlpos = np.flatnonzero(b[chunks[c][1]:size] == 10)
                out[(idx, 1)] = chunks[c][1] + int(nlpos[0]) + 1 if len(nlpos) else size
        res = np.zeros((total, 2), np.int64)
        for (i, k), v in out.items():
            res[i, k] = v
        assert len(out) == 2 * total, (len(out), total)
        return res
    n = total // every_k
    res = np.zeros(n, np.int64)
    for g, v in out.items():
        res[g] = v
    assert len(out) == n
    return res
