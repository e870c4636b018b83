"""CPU restatement of ssszip's gapped container (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` may import this module.  It restates, in plain Python:

* ``encode_vbyte`` / ``decode_vbyte`` -- include/lz77_sss/misc/vbyte.hpp:62-84:
  7 payload bits per byte, least significant group first, bit 7 set on every
  byte but the last;
* ``encode_gapped`` -- cli/ssszip.cpp:119-177: header (1 byte is_64_bit, 8 bytes
  n little endian), then, over the skip_phrases stream, gap records ``{g, 0}``
  and phrases shorter than ``min_lpf_len`` (64, cli/ssszip.cpp:37) that follow a
  gap merge into one gap, flushed before the next written phrase (and at the end)
  as vbyte(length) vbyte(0) + the raw gap bytes; other phrases are written as
  vbyte(i - src) vbyte(len), i = the phrase's text position;
* ``decode_gapped`` -- cli/ssszip.cpp:300-327 (gap records copy raw bytes, others
  copy len bytes from distance src back, byte by byte so overlaps work).

No reference fixture covers this container, so its parity is pinned only by this
restatement and the decode round trip.
"""
from __future__ import annotations

import numpy as np

MIN_LPF_LEN = 64


def encode_vbyte(x: int, out: bytearray) -> None:
    while True:
        b = x & 127
        x >>= 7
        if x:
            b |= 128
        out.append(b)
        if not x:
            return


def decode_vbyte(buf, k: int):
    x, sh = 0, 0
    while True:
        b = buf[k]
        k += 1
        x |= (b & 127) << sh
        sh += 7
        if not b >> 7:
            return x, k


def encode_gapped(stream, text) -> bytes:
    """stream: (k, 2) uint32 skip_phrases records; text: the n input bytes."""
    T = bytes(np.asarray(text, dtype=np.uint8))
    out = bytearray([0])  # is_64_bit = false (pos_t = uint32_t)
    out += len(T).to_bytes(8, "little")
    i, gap, gap_beg, gap_len = 0, False, 0, 0

    def flush():
        encode_vbyte(gap_len, out)
        encode_vbyte(0, out)
        out.extend(T[gap_beg:gap_beg + gap_len])

    for src, ln in np.asarray(stream, dtype=np.uint64).tolist():
        if ln == 0:
            if gap:
                gap_len += src
            else:
                gap_len, gap_beg = src, i
            i += src
            gap = True
        elif gap and ln < MIN_LPF_LEN:
            gap_len += ln
            i += ln
        else:
            if gap:
                flush()
            encode_vbyte(i - src, out)
            encode_vbyte(ln, out)
            i += ln
            gap = False
    if gap:
        flush()
    return bytes(out)


def decode_gapped(buf) -> bytes:
    buf = bytes(buf)
    n = int.from_bytes(buf[1:9], "little")
    out = bytearray()
    k = 9
    while len(out) < n:
        src, k = decode_vbyte(buf, k)
        ln, k = decode_vbyte(buf, k)
        if ln == 0:
            out += buf[k:k + src]
            k += src
        else:
            p = len(out) - src
            if ln <= src:
                out += out[p:p + ln]
            else:
                for t in range(ln):
                    out.append(out[p + t])
    return bytes(out)
