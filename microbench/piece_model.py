"""CPU model of the piece-stream CRC driver (mck_crc_units.hpp crc_pieces_window):
the same slot planning, lane restarts, rotated final shifts and stream-portion
joins, over GF(2) arithmetic, checked against a plain CRC32C.  A design check
run on the CPU before a GPU run; not part of the test suite."""
import random
import sys

POLY = 0x82F63B78


def mulx(a):
    return (a >> 1) ^ (POLY if a & 1 else 0)


def gmul(a, b):
    p = 0
    for j in range(32):
        if b & (0x80000000 >> j):
            p ^= a
        a = mulx(a)
    return p


_pw = {}


def xpow8n(n):
    if n in _pw:
        return _pw[n]
    r, sq, k = 0x80000000, 0x00800000, n
    while k:
        if k & 1:
            r = gmul(r, sq)
        sq = gmul(sq, sq)
        k >>= 1
    _pw[n] = r
    return r


def Z(s, d):
    return gmul(s, xpow8n(d))


def unmulx(b):
    lo = b >> 31
    return (((b ^ (POLY if lo else 0)) << 1) & 0xFFFFFFFF) | lo


def U(s, k):
    for _ in range(8 * k):
        s = unmulx(s)
    return s


def crc32c(init, data):
    c = init ^ 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (POLY if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def words(b16):
    return [int.from_bytes(b16[4 * i:4 * i + 4], "little") for i in range(4)]


def run(buf, spans, W=16, NU=8):
    """spans: list of (off, n, init); returns the CRC list."""
    wn = len(spans)
    out = [None] * wn
    cnt = []
    for off, n, _ in spans:
        a0, a1 = off & ~15, (off + n + 15) & ~15
        cnt.append((a1 - a0) >> 4)
        assert n > 0 and cnt[-1] >= 64
    upre = [0]
    for c in cnt:
        upre.append(upre[-1] + c)
    N = upre[-1]
    T = (N + 63) // 64
    acc = [[0, 0] for _ in range(wn)]

    def span_of(q):  # largest t with upre[t] <= q
        t = 0
        while t + 1 < wn and upre[t + 1] <= q:
            t += 1
        return t

    def load(off, a):
        return bytes(buf[a:a + 16])

    def flush(t, g, es, x, gs, ge):
        p = 0
        for l in range(64):
            r = (l - es) & 63
            p ^= Z(x[l], 4 + 16 * (63 - r))
        off, n, init = spans[t]
        kt = ((off + n + 15) & ~15) - (off + n)
        p0, p1 = upre[t], upre[t + 1]
        if p0 < 64 * gs or p1 > 64 * ge:
            qe = 64 * g + es
            pp = qe - max(p0, 64 * gs)
            p = Z(p, 16 * (p1 - qe))
            acc[t][0] ^= p
            acc[t][1] += pp
            if acc[t][1] != p1 - p0:
                return
            p = acc[t][0]
        if kt:
            p = U(p, kt)
        assert out[t] is None
        out[t] = p ^ 0xFFFFFFFF

    for w in range(W):
        gs, ge = T * w // W, T * (w + 1) // W
        if gs >= ge:
            continue
        s = [0] * 64
        hprev = 0
        for g0 in range(gs, ge, NU):
            plan = []
            for j in range(NU):
                g = g0 + j
                live = g < ge
                q0 = 64 * g
                t = span_of(q0) if live else span_of(min(q0, N - 1))
                p0, p1 = upre[t], upre[t + 1]
                hasn = t < wn - 1
                off, n, init = spans[t]
                e = p1 - q0
                es = e if live and e < 64 else 64
                end = live and (e <= 64 or g + 1 == ge)
                kt = ((off + n + 15) & ~15) - (off + n)
                tail = live and e <= 64 and kt != 0
                heada = live and p0 == q0
                headb = live and e < 64 and hasn
                hl = 0 if heada else (e if headb else 64)
                a0 = off & ~15
                ba = a0 + 16 * (q0 - p0) if live else a0
                offn = spans[t + 1][0] if hasn else off
                bb = ((offn & ~15) if hasn else a0) - 16 * es
                hs = t if heada else t + 1
                plan.append(dict(g=g, t=t, es=es, hl=hl, end=end, tail=tail, head=heada or headb, ba=ba, bb=bb,
                                 kt=kt, hs=hs, first=live and g == gs))
            se = [list(s)]
            for j, P in enumerate(plan):
                new = []
                for l in range(64):
                    a = (P["ba"] if l < P["es"] else P["bb"]) + 16 * l
                    v = bytearray(buf[a:a + 16])
                    extra = 0
                    if P["head"] and l == P["hl"]:
                        hoff, _, hinit = spans[P["hs"]]
                        h0 = hoff & 15
                        for k in range(h0):
                            v[k] = 0
                        extra = U(hinit ^ 0xFFFFFFFF, h0)
                    if P["tail"] and l + 1 == P["es"]:
                        for k in range(16 - P["kt"], 16):
                            v[k] = 0
                    w4 = words(v)
                    restart = P["first"] or l >= P["hl"] or l < hprev
                    x = Z(0 if restart else s[l], 1012) ^ w4[0] ^ extra
                    x = Z(x, 4) ^ w4[1]
                    x = Z(x, 4) ^ w4[2]
                    x = Z(x, 4) ^ w4[3]
                    new.append(x)
                s = new
                se.append(list(s))
                hprev = P["hl"] & 63
            for j, P in enumerate(plan):
                if not P["end"]:
                    continue
                es = P["es"]
                x = [se[j + 1][l] if l < es else se[j][l] for l in range(64)]
                flush(P["t"], P["g"], es, x, gs, ge)
                if P["g"] + 1 == ge and es < 64 and P["hl"] == es:
                    x = [0 if l < es else se[j + 1][l] for l in range(64)]
                    flush(P["t"] + 1, P["g"], 64, x, gs, ge)
    return out


def main():
    rnd = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    for case in range(6):
        nsp = rnd.choice([3, 17, 40, 90])
        lens = []
        for _ in range(nsp):
            k = rnd.random()
            lens.append(rnd.randrange(1009, 1100) if k < 0.3 else rnd.randrange(4096, 4400) if k < 0.8
                        else rnd.randrange(8000, 40000))
        offs, pos = [], rnd.randrange(0, 16)
        for n in lens:
            offs.append(pos)
            pos += n + rnd.choice([0, 0, 4, 5, 33])
        buf = bytes(rnd.getrandbits(8) for _ in range(pos + 64))
        spans = [(o, n, rnd.getrandbits(32) if rnd.random() < 0.3 else 0) for o, n in zip(offs, lens)]
        W = rnd.choice([1, 4, 16])
        NU = rnd.choice([4, 8])
        got = run(buf, spans, W, NU)
        for t, (o, n, init) in enumerate(spans):
            want = crc32c(init, buf[o:o + n])
            assert got[t] == want, (case, t, o, n, W, NU, got[t], want)
        print("case", case, "spans", nsp, "W", W, "NU", NU, "ok")


if __name__ == "__main__":
    main()


def raw(reg, data):
    for b in data:
        reg ^= b
        for _ in range(8):
            reg = (reg >> 1) ^ (POLY if reg & 1 else 0)
    return reg


def run_chunks(buf, spans, W=16, NU=2, layout_base=0):
    """The chunk stream (crc_chunks_window): 64-byte chunks, 4 KiB rounds."""
    wn = len(spans)
    out = [None] * wn
    cnt, info = [], []
    for off, n, init in spans:
        p = layout_base + off
        a1 = (p + n + 15) & ~15
        C = (a1 - p + 63) >> 6
        hb = 64 * C - (a1 - p)
        cnt.append(C)
        info.append(dict(ptr=p, a1=a1, a0=p & ~15, kt=a1 - (p + n), hb=hb, inj=U(init ^ 0xFFFFFFFF, hb), cb=a1 - 64 * C))
        assert a1 - (p & ~15) >= 4096
    upre = [0]
    for c in cnt:
        upre.append(upre[-1] + c)
    N = upre[-1]
    T = (N + 63) // 64
    acc = [[0, 0] for _ in range(wn)]

    def rd(a):
        return bytes(buf[a - layout_base:a - layout_base + 16])

    def span_of(q):
        t = 0
        while t + 1 < wn and upre[t + 1] <= q:
            t += 1
        return t

    def flush(t, g, es, x, gs, ge):
        p = 0
        for l in range(64):
            r = (l - es) & 63
            p ^= Z(x[l], 64 * (63 - r))
        I = info[t]
        p0, p1 = upre[t], upre[t + 1]
        if p0 < 64 * gs or p1 > 64 * ge:
            qe = 64 * g + es
            pp = qe - max(p0, 64 * gs)
            p = Z(p, 64 * (p1 - qe))
            acc[t][0] ^= p
            acc[t][1] += pp
            if acc[t][1] != p1 - p0:
                return
            p = acc[t][0]
        if I["kt"]:
            p = U(p, I["kt"])
        assert out[t] is None
        out[t] = p ^ 0xFFFFFFFF

    for w in range(W):
        gs, ge = T * w // W, T * (w + 1) // W
        if gs >= ge:
            continue
        s = [0] * 64
        hprev = 0
        for g0 in range(gs, ge, NU):
            plan = []
            for j in range(NU):
                g = g0 + j
                live = g < ge
                q0 = 64 * g
                t = span_of(min(q0, N - 1))
                p0, p1 = upre[t], upre[t + 1]
                hasn = t < wn - 1
                I = info[t]
                e = p1 - q0
                es = e if live and e < 64 else 64
                end = live and (e <= 64 or g + 1 == ge)
                tail = live and e <= 64 and I["kt"] != 0
                heada = live and p0 == q0
                headb = live and e < 64 and hasn
                hl = 0 if heada else (e if headb else 64)
                ba = I["cb"] + 64 * (q0 - p0) if live else I["a1"] - 4096
                bb = (info[t + 1]["cb"] if hasn else I["a1"] - 4096) - 64 * es
                H = I if heada else (info[t + 1] if hasn else I)
                plan.append(dict(g=g, t=t, es=es, hl=hl, end=end, tail=tail, head=heada or headb, ba=ba, bb=bb,
                                 kt=I["kt"], H=H, first=live and g == gs))
            se = [list(s)]
            for j, P in enumerate(plan):
                new = []
                for l in range(64):
                    a = (P["ba"] if l < P["es"] else P["bb"]) + 64 * l
                    ch = bytearray()
                    for k in range(4):
                        pa = a + 16 * k
                        if P["head"] and l == P["hl"] and pa < P["H"]["a0"]:
                            pa = P["H"]["a0"]
                        ch += rd(pa)
                    restart = P["first"] or l >= P["hl"] or l < hprev
                    x = 0 if restart else Z(s[l], 4032)
                    if P["head"] and l == P["hl"]:
                        for k in range(P["H"]["hb"]):
                            ch[k] = 0
                        x = P["H"]["inj"]
                    if P["tail"] and l + 1 == P["es"]:
                        for k in range(64 - P["kt"], 64):
                            ch[k] = 0
                    new.append(raw(x, ch))
                s = new
                se.append(list(s))
                hprev = P["hl"] & 63
            for j, P in enumerate(plan):
                if not P["end"]:
                    continue
                es = P["es"]
                x = [se[j + 1][l] if l < es else se[j][l] for l in range(64)]
                flush(P["t"], P["g"], es, x, gs, ge)
                if P["g"] + 1 == ge and es < 64 and P["hl"] == es:
                    x = [0 if l < es else se[j + 1][l] for l in range(64)]
                    flush(P["t"] + 1, P["g"], 64, x, gs, ge)
    return out
