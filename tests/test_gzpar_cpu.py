"""The parallel single-stream inflater (libdpgz dpgz_par_*, csrc/dpgz_par.c) against zlib.

Every case: the inflated bytes equal zlib's, and the access points (offsets, bit positions, member starts,
preceding bytes) and their windows equal those of the zlib-based streaming index (gz.InflateStream), for
several thread counts, region sizes and feed sizes.  Small regions (4-64 KiB) make every batch speculative:
region starts are searched bit by bit, decoded against unknown windows, resolved, and rejected when the
previous region does not end on them.  Corrupt and truncated inputs must raise, never return bytes."""
import gzip
import zlib

import numpy as np
import pytest

from dataplug_amd import gz, synth


def _zlib_ref(blob: bytes, span: int):
    st = gz.InflateStream(span)
    try:
        out = np.zeros(max(64, len(blob) * 1100 // 100 + (1 << 20)), np.uint8)
        c, p, end = st.inflate(blob, True, out, 0, len(out))
        assert end
        pts, win = st.take()
        return out[:p].tobytes(), pts, win
    finally:
        st.close()


def _par(blob: bytes, span: int, threads: int, region: int, step: int):
    pi = gz.ParInflate(span, threads, region_bytes=region)
    try:
        out = bytearray()
        buf = np.zeros(1 << 22, np.uint8)
        pts, wins = [], b""
        i = 0
        while True:
            chunk = blob[i:i + step]
            i += step
            final = i >= len(blob)
            pi.feed(chunk, final)
            while True:
                n = pi.read_into(buf, 0, len(buf))
                if not n:
                    break
                out += buf[:n].tobytes()
            p, w = pi.take(len(out))
            pts.append(p)
            wins += w
            if final:
                break
        st = pi.stats()
        assert st["ended"] == 1 and st["unread"] == 0 and st["points"] == 0
        return bytes(out), np.concatenate(pts), wins, st
    finally:
        pi.close()


def _same(blob, span, threads, region, step):
    exp, epts, ewin = _zlib_ref(blob, span)
    got, gpts, gwin, st = _par(blob, span, threads, region, step)
    assert got == exp
    assert len(gpts) == len(epts)
    for f in epts.dtype.names:
        assert np.array_equal(gpts[f], epts[f]), f
    assert gwin == ewin
    return st


def _deflate(raw: bytes, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, flush_every=0) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, 31, 9, strategy)
    parts = []
    if flush_every:
        for i in range(0, len(raw), flush_every):
            parts.append(c.compress(raw[i:i + flush_every]))
            parts.append(c.flush(zlib.Z_SYNC_FLUSH if (i // flush_every) % 2 else zlib.Z_FULL_FLUSH))
    else:
        parts.append(c.compress(raw))
    parts.append(c.flush())
    return b"".join(parts)


RAW = synth.fastq(9000, seed=11).tobytes()          # ~2 MB of FASTQ


@pytest.mark.parametrize("level", [1, 6, 9])
@pytest.mark.parametrize("threads,region", [(2, 1 << 16), (5, 1 << 14), (8, 1 << 12)])
def test_levels_speculative_regions(level, threads, region):
    st = _same(gzip.compress(RAW, level), 1 << 16, threads, region, 1 << 17)
    assert st["batches"] >= 1


@pytest.mark.parametrize("strategy", [zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FILTERED])
def test_strategies(strategy):
    _same(_deflate(RAW, 6, strategy), 1 << 15, 6, 1 << 13, 300_007)


def test_stored_blocks_and_flushes():
    _same(gzip.compress(RAW[:600_000], 0), 1 << 15, 4, 1 << 13, 1 << 16)           # stored blocks only
    _same(_deflate(RAW, 6, flush_every=77_777), 1 << 15, 6, 1 << 13, 1 << 16)      # sync/full flush points


def test_incompressible_bytes():
    rnd = np.random.default_rng(5).integers(0, 256, 700_000, dtype=np.uint8).tobytes()
    _same(gzip.compress(rnd + RAW[:300_000] + rnd[:100_000], 6), 1 << 15, 8, 1 << 12, 1 << 15)


def test_multi_member_padding_and_tiny_members():
    blob = (gzip.compress(RAW[:700_000], 6) + gzip.compress(b"", 6) + gzip.compress(RAW[700_000:700_010], 9)
            + b"\0" * 9 + gzip.compress(RAW[700_010:], 1) + b"\0" * 3)
    for threads, region, step in [(1, 1 << 20, 1 << 20), (4, 1 << 13, 99_991), (8, 4096, len(blob))]:
        st = _same(blob, 1 << 15, threads, region, step)
        assert st["members"] == 4


def test_header_fields_and_empty_stream():
    import io
    b = io.BytesIO()
    with gzip.GzipFile(filename="reads.fq", mode="wb", fileobj=b, mtime=7) as f:    # FNAME
        f.write(RAW[:200_000])
    _same(b.getvalue(), 1 << 15, 4, 1 << 12, 5000)
    _same(gzip.compress(b""), 1 << 15, 4, 1 << 12, 5000)
    _same(gzip.compress(b"x"), 1 << 15, 4, 1 << 12, 1)


@pytest.mark.parametrize("step", [1, 4093, 65_536])
def test_feed_granularity(step):
    blob = gzip.compress(RAW[:60_000 if step == 1 else 400_000], 6)
    _same(blob, 1 << 14, 3, 1 << 12, step)


def test_corrupt_and_truncated_raise():
    blob = bytearray(gzip.compress(RAW, 6))
    with pytest.raises(ValueError):
        _par(bytes(blob[: len(blob) * 2 // 3]), 1 << 15, 4, 1 << 13, 1 << 16)
    for where in (len(blob) // 5, len(blob) // 2, len(blob) - 12):
        bad = bytearray(blob)
        bad[where:where + 24] = bytes((x ^ 0x5A) for x in bad[where:where + 24])
        with pytest.raises(ValueError):
            _par(bytes(bad), 1 << 15, 4, 1 << 13, 1 << 16)
    bad = bytearray(blob)
    bad[-6] ^= 1                                         # ISIZE
    with pytest.raises(ValueError):
        _par(bytes(bad), 1 << 15, 4, 1 << 13, 1 << 16)
    with pytest.raises(ValueError):
        _par(bytes(blob) + b"garbage!", 1 << 15, 4, 1 << 13, 1 << 16)


def test_many_regions_fuzz():
    """Random slices of FASTQ / CSV text at random levels, region sizes and thread counts."""
    rng = np.random.default_rng(3)
    text = RAW + synth.csv(400_000, 2).tobytes()
    for _ in range(12):
        a = int(rng.integers(0, len(text) // 2))
        b = int(rng.integers(a, len(text)))
        blob = gzip.compress(text[a:b], int(rng.integers(1, 10)))
        _same(blob, int(rng.choice([1 << 12, 1 << 15, 1 << 20])), int(rng.integers(2, 9)),
              int(rng.choice([1024, 4096, 1 << 14])), int(rng.integers(1000, 1 << 18)))
