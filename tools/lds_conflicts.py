"""LDS bank-conflict model of k_scan's three per-byte table reads (class map, D row, K row).

Replays the two reverse automata over synthetic config-2 lanes (64-lane wavefronts, 1 KiB lanes,
resets at utterance starts) and prices every wave-instruction the way MI355X_MICROARCH.md (LDS
section) does for ds_read_b32 / ds_read_u16: two 32-lane groups, one LDS cycle per group, plus one
cycle per extra distinct dword on a bank ((addr/4) mod 32); identical dwords broadcast.
usage: python tools/lds_conflicts.py [n_conv]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
compiler = importlib.import_module("context-based-pii_amd.compiler")
synth = importlib.import_module("context-based-pii_amd.synth")


def lanes_from_corpus(n_conv, lane_bytes=1024):
    bank = synth.build_bank(2048, 2048)
    c = synth.make_corpus(n_conv, 100, bank)
    data, offs = np.asarray(c.data, dtype=np.uint8), np.asarray(c.offsets, dtype=np.int64)
    n = (len(data) // lane_bytes // 64) * 64
    txt = data[: n * lane_bytes].reshape(n, lane_bytes)
    start = np.zeros(len(data) + 1, dtype=bool)
    start[offs[:-1]] = True
    st = start[: n * lane_bytes].reshape(n, lane_bytes)
    return txt, st


def wave_cycles(addr):
    """addr: (L,) byte addresses of one instruction across L lanes (L multiple of 64) -> cycles/wave"""
    dw = (addr >> 2).reshape(-1, 2, 32)
    tot = 0
    for g in range(2):
        d = dw[:, g, :]
        bank = d % 32
        # per group: distinct dwords per bank, max over banks
        key = np.sort(d, axis=1)
        uniq = np.concatenate([np.ones((d.shape[0], 1), bool), key[:, 1:] != key[:, :-1]], axis=1)
        b = np.where(uniq, key % 32, 64)
        cnt = np.zeros((d.shape[0], 65), np.int32)
        np.add.at(cnt, (np.arange(d.shape[0])[:, None], b), 1)
        tot = tot + cnt[:, :32].max(axis=1)
    return tot          # (n_waves,)


def simulate(comp, txt, st, cmap_addr, d_addr, k_addr):
    S = comp.sections
    m = [int(x) for x in S["meta"][:12]]
    SD, CD, d0, SK, CK, k0 = m[4], m[5], m[6], m[7], m[8], m[9]
    td = S["scan.d.trans"].reshape(SD, CD).astype(np.int64)
    tk = S["scan.k.trans"].reshape(SK, CK).astype(np.int64)
    cm = S["scan.cmap2"].astype(np.int64)
    L, B = txt.shape
    sd = np.full(L, d0, np.int64)
    sk = np.full(L, k0, np.int64)
    cyc = np.zeros(3)
    n = 0
    for j in range(B - 1, -1, -1):
        b = txt[:, j].astype(np.int64)
        cc = cm[b]
        cd, ck = cc & 0xFF, cc >> 8
        cyc[0] += wave_cycles(cmap_addr[b]).sum()
        cyc[1] += wave_cycles(d_addr(sd, cd)).sum()
        cyc[2] += wave_cycles(k_addr(sk, ck)).sum()
        n += L // 64
        nd, nk = td[sd, cd] & 0x7FFF, tk[sk, ck] & 0x7FFF
        r = st[:, j]
        sd = np.where(r, d0, nd)
        sk = np.where(r, k0, nk)
    return cyc / n


def main():
    n_conv = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    comp = compiler.compile_default()
    S = comp.sections
    m = [int(x) for x in S["meta"][:12]]
    SD, CD, SK, CK = m[4], m[5], m[7], m[8]
    CDs, CKs = CD + (CD & 1), CK + (CK & 1)
    tk_base = 1024 + SD * CDs * 2
    txt, st = lanes_from_corpus(n_conv)
    print(f"{txt.shape[0]} lanes x {txt.shape[1]} B; D {SD}x{CD}, K {SK}x{CK}")
    cmap_addr = np.arange(256, dtype=np.int64) * 4
    base = simulate(comp, txt, st, cmap_addr, lambda s, c: 1024 + (s * CDs + c) * 2,
                    lambda s, c: tk_base + (s * CKs + c) * 2)
    print("current layout: cycles/wave-instr  cmap %.2f  D %.2f  K %.2f  (conflict-free = 2)" % tuple(base))


if __name__ == "__main__":
    main()


def sweep(n_conv=40):
    comp = compiler.compile_default()
    m = [int(x) for x in comp.sections["meta"][:12]]
    SD, CD, SK, CK = m[4], m[5], m[7], m[8]
    txt, st = lanes_from_corpus(n_conv)
    cmap_addr = np.arange(256, dtype=np.int64) * 4
    for sD in (22, 23, 24, 25, 27, 29, 31, 33):
        for sK in (15, 16, 17, 19, 21, 23):
            kb = 1024 + SD * sD * 4
            r = simulate(comp, txt, st, cmap_addr, lambda s, c: 1024 + s * sD * 4 + c * 2,
                         lambda s, c: kb + s * sK * 4 + c * 2)
            print(f"sD {sD} sK {sK}  LDS {kb + SK * sK * 4:6d} B  cmap {r[0]:.2f} D {r[1]:.2f} K {r[2]:.2f}  sum {r.sum():.2f}")


def heat(comp, txt, st):
    """visit counts of every (row, class) entry of D and K over the lanes"""
    S = comp.sections
    m = [int(x) for x in S["meta"][:12]]
    SD, CD, d0, SK, CK, k0 = m[4], m[5], m[6], m[7], m[8], m[9]
    td = S["scan.d.trans"].reshape(SD, CD).astype(np.int64)
    tk = S["scan.k.trans"].reshape(SK, CK).astype(np.int64)
    cm = S["scan.cmap2"].astype(np.int64)
    L, B = txt.shape
    sd, sk = np.full(L, d0), np.full(L, k0)
    hd, hk = np.zeros((SD, CD)), np.zeros((SK, CK))
    for j in range(B - 1, -1, -1):
        cc = cm[txt[:, j].astype(np.int64)]
        cd, ck = cc & 0xFF, cc >> 8
        np.add.at(hd, (sd, cd), 1)
        np.add.at(hk, (sk, ck), 1)
        nd, nk = td[sd, cd] & 0x7FFF, tk[sk, ck] & 0x7FFF
        r = st[:, j]
        sd, sk = np.where(r, d0, nd), np.where(r, k0, nk)
    return hd, hk


def place_rows(h, Cs, hot_frac=0.995):
    """greedy bank-aware row placement: returns per-row offsets (dwords) and the region size"""
    S, C = h.shape
    w = np.zeros((S, Cs // 2))
    for c in range(C):
        w[:, c // 2] += h[:, c]
    w /= max(w.sum(), 1)
    rows = np.argsort(-w.sum(1))
    cum = np.cumsum(w.sum(1)[rows])
    n_hot = int(np.searchsorted(cum, hot_frac)) + 1
    load = np.zeros(32)
    off = np.zeros(S, np.int64)
    pos = 0
    nd = Cs // 2
    for i, r in enumerate(rows):
        if i < n_hot:
            best, bo = None, 0
            for o in range(32):
                cost = float((w[r] * load[(o + np.arange(nd)) % 32]).sum())
                if best is None or cost < best - 1e-12:
                    best, bo = cost, o
            pad = (bo - pos) % 32
            pos += pad
            load[(pos + np.arange(nd)) % 32] += w[r]
        off[r] = pos
        pos += nd
    return off, pos


def optimized(n_conv=40):
    comp = compiler.compile_default()
    m = [int(x) for x in comp.sections["meta"][:12]]
    SD, CD, SK, CK = m[4], m[5], m[7], m[8]
    CDs, CKs = CD + (CD & 1), CK + (CK & 1)
    txt, st = lanes_from_corpus(n_conv)
    half = txt.shape[0] // 2 // 64 * 64          # train on one half, evaluate on the other
    hd, hk = heat(comp, txt[:half], st[:half])
    for frac in (0.9, 0.99, 0.999):
        od, nD = place_rows(hd, CDs, frac)
        ok, nK = place_rows(hk, CKs, frac)
        kb = 1024 + nD * 4
        cmap_addr = np.arange(256, dtype=np.int64) * 4
        r = simulate(comp, txt[half:], st[half:], cmap_addr, lambda s, c: 1024 + od[s] * 4 + c * 2,
                     lambda s, c: kb + ok[s] * 4 + c * 2)
        print(f"hot {frac}: D {nD * 4} B, K {nK * 4} B: cmap {r[0]:.2f} D {r[1]:.2f} K {r[2]:.2f} sum {r.sum():.2f}")
