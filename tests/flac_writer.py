"""A small FLAC encoder written from the format specification (RFC 9639), test infrastructure only.

libFLAC / libsndfile are absent from the image, so ``mimi_flac_decode`` (csrc/flac.cpp) is checked by round trips:
FLAC is lossless, so a correct decoder must return exactly the PCM this writer encoded -- through every coding
tool the format has (CONSTANT / VERBATIM / FIXED 0-4 / LPC 1-32 subframes, wasted bits, Rice and Rice2
partitions with escape codes, partition orders 0-8, the four channel assignments, fixed and variable block-size
streams, block sizes in the header's 8- and 16-bit fields, sample rates in every header form).  The writer is
independent of the decoder (its own bit writer, CRCs and predictor arithmetic).
"""
import numpy as np


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.nbits = 0

    def put(self, value: int, n: int):
        if n == 0:
            return
        self.acc = (self.acc << n) | (int(value) & ((1 << n) - 1))
        self.nbits += n

    def put_signed(self, value: int, n: int):
        assert -(1 << (n - 1)) <= value < (1 << (n - 1)), (value, n)
        self.put(value & ((1 << n) - 1), n)

    def unary(self, q: int):  # q zeros, then a one
        self.put(1, q + 1)

    def align(self):
        if self.nbits % 8:
            self.put(0, 8 - self.nbits % 8)

    def bytes(self) -> bytes:
        assert self.nbits % 8 == 0
        return self.acc.to_bytes(self.nbits // 8, "big") if self.nbits else b""


def crc8(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def coded_number(v: int) -> bytes:
    """The frame / sample number in the UTF-8-like form (1-7 bytes, up to 36 bits)."""
    if v < 0x80:
        return bytes([v])
    for n in range(2, 8):
        if v < (1 << (5 * n + 1 if n < 7 else 36)):
            out = []
            for _ in range(n - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            lead = (0xFF << (8 - n)) & 0xFF
            return bytes([lead | v] + out[::-1])
    raise ValueError(v)


def _zigzag(r: int) -> int:
    return (r << 1) if r >= 0 else ((-r) << 1) - 1


def _fixed_residual(s, order):
    s = [int(v) for v in s]
    res = []
    for i in range(order, len(s)):
        if order == 0:
            p = 0
        elif order == 1:
            p = s[i - 1]
        elif order == 2:
            p = 2 * s[i - 1] - s[i - 2]
        elif order == 3:
            p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]
        else:
            p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]
        res.append(s[i] - p)
    return res


def _lpc_coefs(s, order, precision, rng):
    """Quantised predictor coefficients (least squares on the block, or random when degenerate) and a shift."""
    x = np.asarray(s, dtype=np.float64)
    n = len(x)
    if n > order + 4 and np.any(x != x[0]):
        A = np.stack([x[order - 1 - j:n - 1 - j] for j in range(order)], axis=1)  # column j: sample j + 1 back
        c, *_ = np.linalg.lstsq(A, x[order:], rcond=None)
    else:
        c = rng.uniform(-1, 1, order)
    cmax = float(np.max(np.abs(c))) if order else 0.0
    lim = (1 << (precision - 1)) - 1
    shift = 0
    while shift < 15 and cmax * (1 << (shift + 1)) <= lim:
        shift += 1
    q = np.clip(np.round(c * (1 << shift)), -lim - 1, lim).astype(np.int64)
    return [int(v) for v in q], shift


def _lpc_residual(s, coefs, shift):
    s = [int(v) for v in s]
    order = len(coefs)
    res = []
    for i in range(order, len(s)):
        acc = 0
        for j, c in enumerate(coefs):
            acc += c * s[i - 1 - j]
        res.append(s[i] - (acc >> shift))
    return res


def _write_residual(bw: BitWriter, res, bs, order, porder, rng, escape_prob=0.1):
    parts = 1 << porder
    psize = bs >> porder
    zz = [_zigzag(r) for r in res]
    # Rice2 (5-bit parameters) whenever a partition wants a parameter above 14, else Rice (4 bits)
    chunks, i = [], 0
    for p in range(parts):
        cnt = psize - order if p == 0 else psize
        chunks.append((res[i:i + cnt], zz[i:i + cnt]))
        i += cnt
    best = []
    for r, z in chunks:
        mean = (sum(z) / len(z)) if z else 0
        k = max(0, int(np.floor(np.log2(mean + 1))) if mean > 0 else 0)
        best.append(k)
    method = 1 if max(best + [0]) > 14 or rng.random() < 0.3 else 0
    pbits = 4 if method == 0 else 5
    esc = (1 << pbits) - 1
    bw.put(method, 2)
    bw.put(porder, 4)
    for (r, z), k in zip(chunks, best):
        k = min(k, esc - 1)
        if r and rng.random() < escape_prob:
            nb = max(int(abs(v)).bit_length() + 1 for v in r)
            if nb <= 31:
                bw.put(esc, pbits)
                bw.put(nb, 5)
                for v in r:
                    bw.put_signed(v, nb)
                continue
        if not r and rng.random() < 0.5:  # an empty escape partition: 0 bits per sample
            bw.put(esc, pbits)
            bw.put(0, 5)
            continue
        bw.put(k, pbits)
        for v in z:
            bw.unary(v >> k)
            bw.put(v & ((1 << k) - 1), k)


def _write_subframe(bw: BitWriter, s, bps, kind, rng):
    """kind: 'constant', 'verbatim', ('fixed', order), ('lpc', order, precision)."""
    s = [int(v) for v in s]
    bs = len(s)
    wasted = 0
    if any(s) and rng.random() < 0.5:
        while wasted < bps - 1 and all(v % (1 << (wasted + 1)) == 0 for v in s):
            wasted += 1
    b = bps - wasted
    t = [v >> wasted for v in s]
    name = kind if isinstance(kind, str) else kind[0]
    bw.put(0, 1)
    if name == "constant":
        bw.put(0, 6)
    elif name == "verbatim":
        bw.put(1, 6)
    elif name == "fixed":
        bw.put(8 + kind[1], 6)
    else:
        bw.put(32 + kind[1] - 1, 6)
    if wasted:
        bw.put(1, 1)
        bw.unary(wasted - 1)
    else:
        bw.put(0, 1)
    if name == "constant":
        bw.put_signed(t[0], b)
    elif name == "verbatim":
        for v in t:
            bw.put_signed(v, b)
    else:
        order = kind[1]
        for v in t[:order]:
            bw.put_signed(v, b)
        if name == "fixed":
            res = _fixed_residual(t, order)
        else:
            precision = kind[2]
            coefs, shift = _lpc_coefs(t, order, precision, rng)
            bw.put(precision - 1, 4)
            bw.put_signed(shift, 5)
            for c in coefs:
                bw.put_signed(c, precision)
            res = _lpc_residual(t, coefs, shift)
        max_po = 0
        while max_po < 8 and bs % (1 << (max_po + 1)) == 0 and (bs >> (max_po + 1)) >= order:
            max_po += 1
        porder = int(rng.integers(0, max_po + 1))
        _write_residual(bw, res, bs, order, porder, rng)


_BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
             8192: 13, 16384: 14, 32768: 15}
_RATE_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
               48000: 10, 96000: 11}
_BPS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def encode(pcm: np.ndarray, rate: int, bps: int, block_sizes=None, seed: int = 0, kinds=None,
           variable: bool = False, header_rate: bool = None, id3: bool = False, total_known: bool = True) -> bytes:
    """pcm: int [channels, n].  Returns a FLAC file.  Each frame draws its subframe kinds, channel assignment and
    coding choices from ``seed``; ``block_sizes`` (a list, cycled) sets the frame lengths."""
    rng = np.random.default_rng(seed)
    pcm = np.asarray(pcm, dtype=np.int64)
    C, n = pcm.shape
    assert 1 <= C <= 8 and 4 <= bps <= 32
    block_sizes = list(block_sizes or [4096])
    kinds = kinds or ["constant", "verbatim", ("fixed", 0), ("fixed", 1), ("fixed", 2), ("fixed", 3), ("fixed", 4),
                      ("lpc", 1, 12), ("lpc", 4, 15), ("lpc", 8, 14), ("lpc", 12, 13), ("lpc", 32, 15),
                      ("lpc", 2, 5)]
    out = bytearray()
    if id3:
        body = b"TIT2\x00\x00\x00\x05\x00\x00\x03abcd"
        sz = len(body)
        out += b"ID3\x04\x00\x00" + bytes([(sz >> 21) & 0x7F, (sz >> 14) & 0x7F, (sz >> 7) & 0x7F, sz & 0x7F]) + body
    out += b"fLaC"
    si = BitWriter()
    si.put(min(block_sizes) if not variable else 16, 16)
    si.put(max(block_sizes), 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(rate, 20)
    si.put(C - 1, 3)
    si.put(bps - 1, 5)
    si.put(n if total_known else 0, 36)
    si.put(0, 128)
    # a PADDING block after STREAMINFO, then the last-block flag on it
    out += bytes([0x00, 0, 0, 34]) + si.bytes()
    out += bytes([0x81, 0, 0, 7]) + bytes(7)
    pos, fno, bi = 0, 0, 0
    while pos < n:
        bs = min(block_sizes[bi % len(block_sizes)], n - pos)
        bi += 1
        blk = pcm[:, pos:pos + bs]
        hdr = BitWriter()
        hdr.put(0b11111111111110, 14)
        hdr.put(0, 1)
        hdr.put(1 if variable else 0, 1)
        if bs in _BS_CODES and rng.random() < 0.8:
            bcode, bextra = _BS_CODES[bs], None
        elif bs <= 256:
            bcode, bextra = 6, (bs - 1, 8)
        else:
            bcode, bextra = 7, (bs - 1, 16)
        hdr.put(bcode, 4)
        use_hdr_rate = header_rate if header_rate is not None else (fno % 3 != 0)
        rextra = None
        if not use_hdr_rate:
            rcode = 0
        elif rate in _RATE_CODES and fno % 2 == 0:
            rcode = _RATE_CODES[rate]
        elif rate % 1000 == 0 and rate // 1000 < 256:
            rcode, rextra = 12, (rate // 1000, 8)
        elif rate < 65536:
            rcode, rextra = 13, (rate, 16)
        else:
            rcode, rextra = 14, (rate // 10, 16)
        hdr.put(rcode, 4)
        # channel assignment: independent, or a stereo decorrelation (whichever the draw picks)
        chan = 0
        if C == 2:
            chan = int(rng.choice([1, 8, 9, 10]))
        hdr.put(C - 1 if chan in (0, 1) else chan, 4)
        hdr.put(_BPS_CODES.get(bps, 0) if fno % 2 else 0, 3)
        hdr.put(0, 1)
        hdr.align()
        head = hdr.bytes() + coded_number(pos if variable else fno)
        tail = BitWriter()
        if bextra:
            tail.put(*bextra)
        if rextra:
            tail.put(*rextra)
        head += tail.bytes()
        head += bytes([crc8(head)])
        # subframes
        L, R = (blk[0], blk[1]) if C == 2 else (None, None)
        if C == 2 and chan == 8:
            chans = [(L, bps), (L - R, bps + 1)]
        elif C == 2 and chan == 9:
            chans = [(L - R, bps + 1), (R, bps)]
        elif C == 2 and chan == 10:
            chans = [((L + R) >> 1, bps), (L - R, bps + 1)]
        else:
            chans = [(blk[c], bps) for c in range(C)]
        body = BitWriter()
        for s, b in chans:
            if np.all(s == s[0]) and rng.random() < 0.7:
                kind = "constant"
            else:
                kind = kinds[int(rng.integers(0, len(kinds)))]
                if kind == "constant" and not np.all(s == s[0]):
                    kind = "verbatim"
                name = kind if isinstance(kind, str) else kind[0]
                if name in ("fixed", "lpc") and kind[1] > bs:
                    kind = "verbatim"
            _write_subframe(body, s, b, kind, rng)
        body.align()
        frame = head + body.bytes()
        frame += crc16(frame).to_bytes(2, "big")
        out += frame
        pos += bs
        fno += 1
    return bytes(out)
