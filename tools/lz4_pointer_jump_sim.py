"""Would pointer jumping resolve LZ4 match bytes in parallel?

For a batch of B output bytes, every match byte x points at its source
x - off; a source inside the batch that is itself a match byte points on.
Repeated doubling (ptr = ptr[ptr]) resolves every byte to a literal byte
or to history before the batch in ceil(log2(chain depth)) rounds, each a
lane-parallel LDS gather — instead of copying the batch's matches one by
one (the serial part of every few-stream decoder here).  This replays
pyarrow LZ4 frames on the CPU and reports, per batch size, the rounds
needed (max / mean over batches) and the chain depth.

``python tools/lz4_pointer_jump_sim.py``
"""
import struct
import sys

import numpy as np

sys.path.insert(0, ".")


def sequences(block: bytes):
    q, e, out = 0, len(block), []
    while q < e:
        t = block[q]
        q += 1
        lit, ml = t >> 4, t & 15
        if lit == 15:
            while True:
                x = block[q]
                q += 1
                lit += x
                if x != 255:
                    break
        q += lit
        if q >= e:
            out.append((lit, 0, 0))
            break
        off = block[q] | block[q + 1] << 8
        q += 2
        if ml == 15:
            while True:
                x = block[q]
                q += 1
                ml += x
                if x != 255:
                    break
        out.append((lit, off, ml + 4))
    return out


def frame_blocks(f: bytes):
    from nvme_strom_amd.ops import decompress as D
    info = D.parse_lz4_frame_header(f)
    p, out = info.data_offset, []
    while True:
        bs, = struct.unpack_from("<I", f, p)
        p += 4
        if bs == 0:
            return out
        stored = bs >> 31
        bs &= 0x7FFFFFFF
        out.append((stored, f[p:p + bs]))
        p += bs + (4 if info.block_checksum else 0)


def rounds_for(seqs, total, batch):
    src = np.full(total, -1, dtype=np.int64)          # -1: literal byte
    x = 0
    for lit, off, m in seqs:
        x += lit
        if m:
            k = np.arange(m)
            # overlapping copies: byte k repeats byte k mod off
            src[x:x + m] = x - off + (k % off)
            x += m
    res = []
    for b0 in range(0, total, batch):
        p = src[b0:b0 + batch].copy()
        idx = np.arange(b0, b0 + len(p))
        r = 0
        while True:
            inside = (p >= b0) & (p >= 0)
            nxt = np.where(inside, src[np.clip(p, 0, total - 1)], -2)
            # a pointer is final once it reaches a literal (-1) or history (< b0)
            move = inside & (nxt != -1)
            if not move.any():
                break
            p = np.where(move, nxt, p)
            r += 1
        res.append(r)
    return res


def main():
    import pyarrow as pa
    rng = np.random.default_rng(3)
    words = [b"select", b"from", b"where", b"gpu", b"hbm", b"nvme", b"strom", b"table"]
    corpora = {
        "val (config 5)": rng.integers(0, 1_000_000, 65536, dtype=np.int64).tobytes(),
        "sorted ids": np.cumsum(rng.integers(0, 4096, 65536)).astype(np.int64).tobytes(),
        "text": b" ".join(words[i] for i in rng.integers(0, len(words), 120000))[:512 << 10],
    }
    for name, raw in corpora.items():
        f = pa.compress(raw, codec="lz4", asbytes=True)
        seqs = []
        for stored, blk in frame_blocks(f):
            seqs += [(len(blk), 0, 0)] if stored else sequences(blk)
        for batch in (1024, 4096, 16384):
            r = rounds_for(seqs, len(raw), batch)
            # plain jumping is linear in the chain; doubling is log2 of it
            depth = max(r)
            print(f"{name:16s} batch {batch:6d}: chain depth max {depth:5d} mean {np.mean(r):7.1f}"
                  f"  doubling rounds <= {int(np.ceil(np.log2(depth + 1)))}")


if __name__ == "__main__":
    main()
