"""Seeded synthetic objects for tests and the benchmark (FASTA / CSV / VCF / FASTQ).

Every generator returns a ``numpy.uint8`` array of EXACTLY the requested size (or read count) and
is deterministic for a given ``seed`` on a given numpy version (tests pin the bytes with a sha256).
The shapes follow the reference's sample data and BASELINE.json configs:

* FASTA: ``>seq{i} synthetic record len={L}\\n`` headers, L uniform in [1000, 3000), 60-column
  ACGT lines.  The object never ends inside a header line, so the reference's
  uint32 index stays defined at exactly 4 GiB.
* CSV:   cities.csv row shape (10 columns, ``int,int,int,N,int,int,int,W,City,ST\\n``).
* VCF:   a VCFv4 header + 12 tab-separated columns per row.
* FASTQ: 4-line reads, ``@id / SEQ / + / QUAL``, fixed read length.

Large objects are built by :func:`tile_plan`: one seeded base block of a length that is NOT a power
of two, repeated, so that kernel tile boundaries fall at a different phase in every copy.
"""
from __future__ import annotations

import hashlib

import numpy as np

_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_QUAL = np.frombuffer(b"!#$%&'()*+,-./0123456789:;<=>?@ABCDEFGHIJ", dtype=np.uint8)


def sha256(a) -> str:
    return hashlib.sha256(memoryview(np.ascontiguousarray(a)).cast("B")).hexdigest()


def _scatter_strings(out: np.ndarray, starts: np.ndarray, blob: np.ndarray, lens: np.ndarray) -> None:
    """out[starts[i] : starts[i]+lens[i]] = i-th string of the concatenated ``blob``."""
    if len(lens) == 0:
        return
    seg_start = np.repeat(starts - np.concatenate(([0], np.cumsum(lens)[:-1])), lens)
    idx = seg_start + np.arange(int(lens.sum()), dtype=np.int64)
    out[idx] = blob


def fasta(size: int, seed: int = 0, line_width: int = 60, seq_min: int = 1000, seq_max: int = 3000,
          first_id: int = 0) -> np.ndarray:
    """A FASTA object of exactly ``size`` bytes."""
    if size <= 0:
        return np.zeros(0, np.uint8)
    rng = np.random.default_rng(seed)
    avg = 40 + (seq_min + seq_max) / 2 * (1 + 1 / line_width)
    n = int(size / avg * 1.1) + 4
    L = rng.integers(seq_min, seq_max, n).astype(np.int64)
    headers = [f">seq{first_id + i} synthetic record len={int(l)}\n".encode() for i, l in enumerate(L)]
    hl = np.fromiter((len(h) for h in headers), dtype=np.int64, count=n)
    nlines = (L + line_width - 1) // line_width
    rec = hl + L + nlines
    ends = np.cumsum(rec)
    n = int(np.searchsorted(ends, size)) + 1            # records needed to cover ``size``
    L, hl, nlines, rec = L[:n], hl[:n], nlines[:n], rec[:n]
    total = int(rec.sum())
    starts = np.concatenate(([0], np.cumsum(rec)[:-1]))
    out = _ACGT[rng.integers(0, 4, total, dtype=np.uint8)]
    _scatter_strings(out, starts, np.frombuffer(b"".join(headers[:n]), np.uint8), hl)
    # newline after every ``line_width`` bases and after the last (partial) line of each record
    body = starts + hl
    k = np.arange(int(nlines.sum()), dtype=np.int64) - np.repeat(np.cumsum(nlines) - nlines, nlines)
    nl = np.repeat(body, nlines) + np.minimum((k + 1) * (line_width + 1) - 1,
                                              np.repeat(L + nlines - 1, nlines))
    out[nl] = 10
    out = out[:size].copy()
    _fix_fasta_tail(out)
    return out


def _fix_fasta_tail(a: np.ndarray) -> None:
    """Never end inside a header line (keeps every reference ``end`` < size, i.e. uint32-safe)."""
    nls = np.flatnonzero(a == 10)
    tail0 = int(nls[-1]) + 1 if len(nls) else 0
    if tail0 < len(a) and (a[tail0:] == ord(">")).any():
        a[tail0:] = ord("N")


_CITIES = [b"Youngstown,OH", b"Yankton,SD", b"Yakima,WA", b"Worcester,MA", b"Wisconsin Dells,WI",
           b"Winston-Salem,NC", b"Wilmington,DE", b"Williston,ND", b"Wichita Falls,TX", b"Wheeling,WV",
           b"Waterloo,IA", b"Salt Lake City,UT", b"San Antonio,TX", b"Sacramento,CA", b"Ravenna,OH"]
CSV_HEADER = b"LatD,LatM,LatS,NS,LonD,LonM,LonS,EW,City,State\n"


def csv(size: int, seed: int = 0) -> np.ndarray:
    """A cities.csv-shaped CSV object of exactly ``size`` bytes (ends with ``\\n``)."""
    rng = np.random.default_rng(seed)
    rows = [CSV_HEADER]
    total = len(CSV_HEADER)
    while total < size:
        m = 4096
        v = rng.integers(0, 60, (m, 6))
        ci = rng.integers(0, len(_CITIES), m)
        for j in range(m):
            r = b"%d,%d,%d,N,%d,%d,%d,W,%s\n" % (v[j, 0] % 50 + 25, v[j, 1], v[j, 2], v[j, 3] + 60,
                                                  v[j, 4], v[j, 5], _CITIES[ci[j]])
            rows.append(r)
            total += len(r)
    out = np.frombuffer(b"".join(rows), np.uint8)[:size].copy()
    if size:
        out[-1] = 10
    return out


def csv_wide(size: int, seed: int = 0, max_note: int = 1500) -> np.ndarray:
    """``csv`` rows with an 11th column ``Note`` of 0..max_note ASCII characters: rows longer than the
    reference's default slice padding (256 B), which reach CSVSlice.get's buffer expansion (csv.py:81-94)."""
    base = csv(size, seed).tobytes().split(b"\n")[1:-1]
    rng = np.random.default_rng(seed + 1)
    rows = [CSV_HEADER[:-1] + b",Note\n"]
    total = len(rows[0])
    i = 0
    while total < size:
        r = base[i % len(base)] + b"," + b"n" * int(rng.integers(0, max_note + 1)) + b"\n"
        rows.append(r)
        total += len(r)
        i += 1
    out = np.frombuffer(b"".join(rows), np.uint8)[:size].copy()
    if size:
        out[-1] = 10
    return out


VCF_HEADER = (b"##fileformat=VCFv4.2\n"
              b"##source=dataplug_amd.synth\n"
              b"##INFO=<ID=NS,Number=1,Type=Integer,Description=\"Samples With Data\">\n"
              b"##INFO=<ID=DP,Number=1,Type=Integer,Description=\"Total Depth\">\n"
              b"##INFO=<ID=AF,Number=A,Type=Float,Description=\"Allele Frequency\">\n"
              b"##FILTER=<ID=q10,Description=\"Quality below 10\">\n"
              b"##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
              b"##FORMAT=<ID=GQ,Number=1,Type=Integer,Description=\"Genotype Quality\">\n"
              b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\tS2\tS3\n")


def vcf(size: int, seed: int = 0) -> np.ndarray:
    """A VCF object of exactly ``size`` bytes: header + 12-column rows (ends with ``\\n``)."""
    rng = np.random.default_rng(seed)
    rows = [VCF_HEADER]
    total = len(VCF_HEADER)
    pos = 1000
    gts = [b"0|0", b"0|1", b"1|0", b"1/1", b"./."]
    while total < size:
        m = 4096
        v = rng.integers(0, 1 << 30, (m, 8))
        for j in range(m):
            pos += int(v[j, 0] % 500) + 1
            r = b"%d\t%d\trs%d\t%c\t%c\t%d\tPASS\tNS=3;DP=%d;AF=0.%d\tGT:GQ\t%s:%d\t%s:%d\t%s:%d\n" % (
                int(v[j, 1] % 22) + 1, pos, int(v[j, 2] % 10**7), b"ACGT"[v[j, 3] % 4], b"ACGT"[v[j, 4] % 4],
                int(v[j, 5] % 99), int(v[j, 6] % 40), int(v[j, 7] % 1000),
                gts[v[j, 1] % 5], int(v[j, 2] % 60), gts[v[j, 3] % 5], int(v[j, 4] % 60),
                gts[v[j, 5] % 5], int(v[j, 6] % 60))
            rows.append(r)
            total += len(r)
    out = np.frombuffer(b"".join(rows), np.uint8)[:size].copy()
    if size:
        out[-1] = 10
    return out


def vcf_wide(size: int, seed: int = 0, max_info: int = 1500) -> np.ndarray:
    """``vcf`` rows whose INFO field carries an extra ``NOTE=`` of 0..max_info characters: rows longer than
    the slice padding, which reach VCFSlice.get's range expansion (vcf.py:117-136)."""
    base = vcf(size, seed).tobytes()
    head_end = base.index(b"\n#CHROM") + 1
    head_end = base.index(b"\n", head_end) + 1
    body = base[head_end:].split(b"\n")[:-1]
    rng = np.random.default_rng(seed + 1)
    rows = [base[:head_end]]
    total = len(rows[0])
    i = 0
    while total < size:
        f = body[i % len(body)].split(b"\t")
        if len(f) >= 8:
            f[7] = f[7] + b";NOTE=" + b"v" * int(rng.integers(0, max_info + 1))
        r = b"\t".join(f) + b"\n"
        rows.append(r)
        total += len(r)
        i += 1
    out = np.frombuffer(b"".join(rows), np.uint8)[:size].copy()
    if size:
        out[-1] = 10
    return out


def fastq(n_reads: int, seed: int = 0, read_len: int = 100) -> np.ndarray:
    """``n_reads`` 4-line FASTQ reads (inflated stream)."""
    rng = np.random.default_rng(seed)
    ids = [b"@read%d synthetic/1\n" % i for i in range(n_reads)]
    il = np.fromiter((len(h) for h in ids), np.int64, count=n_reads)
    rec = il + (read_len + 1) + 2 + (read_len + 1)
    starts = np.concatenate(([0], np.cumsum(rec)[:-1])).astype(np.int64)
    total = int(rec.sum())
    out = np.empty(total, np.uint8)
    _scatter_strings(out, starts, np.frombuffer(b"".join(ids), np.uint8), il)
    seq0 = starts + il
    j = np.arange(read_len, dtype=np.int64)
    out[(seq0[:, None] + j).ravel()] = _ACGT[rng.integers(0, 4, n_reads * read_len, dtype=np.uint8)]
    out[seq0 + read_len] = 10
    out[seq0 + read_len + 1] = ord("+")
    out[seq0 + read_len + 2] = 10
    q0 = seq0 + read_len + 3
    out[(q0[:, None] + j).ravel()] = _QUAL[rng.integers(0, len(_QUAL), n_reads * read_len, dtype=np.uint8)]
    out[q0 + read_len] = 10
    return out


def tile_plan(block_len: int, size: int):
    """Copies of a base block that fill ``size`` bytes: list of (dst_offset, length)."""
    plan, off = [], 0
    while off < size:
        n = min(block_len, size - off)
        plan.append((off, n))
        off += n
    return plan


def tiled_fasta_host(size: int, seed: int = 0, block: int = 64 * 2**20 - 4099) -> np.ndarray:
    """Host-side FASTA of exactly ``size`` bytes made of repeated seeded blocks (tail-fixed)."""
    base = fasta(min(block, size), seed)
    out = np.empty(size, np.uint8)
    for off, n in tile_plan(len(base), size):
        out[off:off + n] = base[:n]
    _fix_fasta_tail(out)
    return out


class TiledFasta:
    """``tiled_fasta_host(size, seed)`` without materializing it: any byte range on demand.

    The multi-GPU benchmark indexes ONE object of N x 4 GiB whose chunk groups live on different GPUs; each
    worker builds only the bytes of its own group (plus the look-ahead halo).  ``bytes_range(0, size)``
    equals ``tiled_fasta_host(size, seed)`` byte for byte (tests/test_synth_tiled.py)."""

    def __init__(self, size: int, seed: int = 0, block: int = 64 * 2**20 - 4099):
        self.size = int(size)
        self.base = fasta(min(block, self.size), seed)
        # the object-level tail fix of _fix_fasta_tail: bytes after the object's last '\n'
        t0 = max(0, self.size - (1 << 20))
        tail = self._raw(t0, self.size)
        nls = np.flatnonzero(tail == 10)
        self.tail0 = t0 + int(nls[-1]) + 1 if len(nls) else 0
        self.tail_fix = self.tail0 < self.size and bool((tail[self.tail0 - t0:] == ord(">")).any())

    def _raw(self, start: int, end: int, out: np.ndarray | None = None) -> np.ndarray:
        out = np.empty(end - start, np.uint8) if out is None else out[: end - start]
        bl = len(self.base)
        p = start
        while p < end:
            q = p % bl
            n = min(bl - q, end - p)
            out[p - start:p - start + n] = self.base[q:q + n]
            p += n
        return out

    def bytes_range(self, start: int, end: int, out: np.ndarray | None = None) -> np.ndarray:
        out = self._raw(start, end, out)
        if self.tail_fix and end > self.tail0:
            out[max(self.tail0, start) - start:] = ord("N")
        return out


def tiled_host(base: np.ndarray, size: int) -> np.ndarray:
    """``size`` bytes made of repeated copies of ``base`` (the last copy truncated)."""
    out = np.empty(size, np.uint8)
    for off, n in tile_plan(len(base), size):
        out[off:off + n] = base[:n]
    return out


class TiledText:
    """A large line-oriented object: ``head`` once, then ``body`` repeated to exactly ``size`` bytes.

    Used for the BASELINE configs[2]/[3] shapes (32 GiB CSV, 64 GiB VCF): a rank materializes only the
    byte range it scans (:meth:`bytes_range`), and the expected newline offsets of any range follow from
    the body's own newlines (:meth:`delims_range`), so a multi-GiB index is checked without a second scan.
    """

    def __init__(self, head: np.ndarray, body: np.ndarray, size: int, delim: int = 10):
        self.head = np.ascontiguousarray(head, np.uint8)
        self.body = np.ascontiguousarray(body, np.uint8)
        self.size = int(size)
        self.delim = delim
        self.head_pos = np.flatnonzero(self.head == delim).astype(np.uint64)
        self.body_pos = np.flatnonzero(self.body == delim).astype(np.uint64)

    def _tiles(self, start: int, end: int):
        """(object offset, body offset, length) pieces of the body covering [start, end)."""
        h, bl = len(self.head), len(self.body)
        p = max(start, h)
        while p < end:
            q = (p - h) % bl
            n = min(bl - q, end - p)
            yield p, q, n
            p += n

    def bytes_range(self, start: int, end: int, out: np.ndarray | None = None) -> np.ndarray:
        out = np.empty(end - start, np.uint8) if out is None else out[: end - start]
        h = len(self.head)
        if start < h:
            out[: min(h, end) - start] = self.head[start:min(h, end)]
        for p, q, n in self._tiles(start, end):
            out[p - start:p - start + n] = self.body[q:q + n]
        return out

    def delims_range(self, start: int, end: int):
        """Yields sorted uint64 arrays: the delimiter offsets in [start, end), piece by piece."""
        h = len(self.head)
        if start < h:
            hp = self.head_pos
            yield hp[(hp >= start) & (hp < min(h, end))]
        bp = self.body_pos
        for p, q, n in self._tiles(start, end):
            lo, hi = np.searchsorted(bp, q), np.searchsorted(bp, q + n)
            yield bp[lo:hi] + np.uint64(p - q)

    def count_range(self, start: int, end: int) -> int:
        return int(sum(len(x) for x in self.delims_range(start, end)))


def tiled_csv(size: int, seed: int = 0, block: int = 64 * 2**20 - 333) -> TiledText:
    """cities.csv-shaped CSV of ``size`` bytes: one header line, then a seeded row block repeated."""
    base = csv(block, seed)
    h = len(CSV_HEADER)
    return TiledText(base[:h], base[h:], size)


def tiled_vcf(size: int, seed: int = 0, block: int = 64 * 2**20 - 333) -> TiledText:
    """VCF of ``size`` bytes: the header once, then a seeded row block repeated."""
    base = vcf(block, seed)
    h = len(VCF_HEADER)
    return TiledText(base[:h], base[h:], size)


def bgzf(raw: bytes, block: int = 65280, level: int = 6, eof: bool = True) -> bytes:
    """BGZF (blocked gzip, as samtools/htslib write FASTQ.gz): independent gzip members of at most ``block``
    inflated bytes, each carrying its compressed size in the "BC" extra subfield, plus the empty EOF member."""
    import struct
    import zlib
    out = []

    def member(data: bytes) -> bytes:
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(data) + c.flush()
        bsize = 18 + len(body) + 8 - 1
        head = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff" + struct.pack("<H", 6) + b"BC" + \
            struct.pack("<HH", 2, bsize)
        return head + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF)

    for i in range(0, len(raw), block):
        out.append(member(raw[i:i + block]))
    if eof:
        out.append(member(b""))
    return b"".join(out)
