// pii_device.h - per-lane building blocks of the scan-and-redact pipeline (gfx950).
//
// Validators restate SURVEY.md Appendix A.1 / oracle/pii_oracle.py (v_luhn ... v_iban) as forward
// single-pass byte machines; the DFA runners execute the tables built by
// context-based-pii_amd/compiler.py.  Text is read through 16-byte windows assembled from aligned
// 16-byte loads (never a byte load per step, never a chunk outside the bytes asked for).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pii {

// character kinds used by the DFA start states (compiler.K_BOT/K_W/K_N)
enum { K_BOT = 0, K_W = 1, K_N = 2 };

__device__ __forceinline__ bool is_word(uint32_t c) {
    return (c - '0' < 10u) | ((c | 32u) - 'a' < 26u) | (c == '_');
}
__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }

// ---------------------------------------------------------------------------------- text windows
// 16 bytes starting at byte o (0..15) of the 32-byte window {a, b}
__device__ __forceinline__ uint4 window16(const uint4& a, const uint4& b, uint32_t o) {
    const uint32_t d = o >> 2, s = o & 3;
    const uint32_t w0 = a.x, w1 = a.y, w2 = a.z, w3 = a.w, w4 = b.x, w5 = b.y, w6 = b.z, w7 = b.w;
    const uint32_t v0 = d == 0 ? w0 : d == 1 ? w1 : d == 2 ? w2 : w3;
    const uint32_t v1 = d == 0 ? w1 : d == 1 ? w2 : d == 2 ? w3 : w4;
    const uint32_t v2 = d == 0 ? w2 : d == 1 ? w3 : d == 2 ? w4 : w5;
    const uint32_t v3 = d == 0 ? w3 : d == 1 ? w4 : d == 2 ? w5 : w6;
    const uint32_t v4 = d == 0 ? w4 : d == 1 ? w5 : d == 2 ? w6 : w7;
    return make_uint4(__builtin_amdgcn_alignbyte(v1, v0, s), __builtin_amdgcn_alignbyte(v2, v1, s),
                      __builtin_amdgcn_alignbyte(v3, v2, s), __builtin_amdgcn_alignbyte(v4, v3, s));
}

// bytes [src, src + 16) as a uint4, reading only the aligned 16-byte chunks that hold a byte of
// [src + need_lo, src + need_hi) (so never a chunk outside the caller's buffer); other bytes are 0
// Every caller passes a pointer into HBM (text, token bytes, window rings): the loads are issued as
// global (address space 1), not flat -- a flat load also counts against lgkmcnt, so the next LDS
// wait would stall on it.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4_t g_u32x4_t;
__device__ __forceinline__ uint4 gload16(uintptr_t a) {      // 16-byte aligned global load
    const u32x4_t v = *(g_u32x4_t*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
// the same at a uniform base + a 32-bit byte offset (the SGPR-base addressing form)
__device__ __forceinline__ uint4 gload16_at(const uint8_t* base, uint32_t off) {
    const u32x4_t v = *(g_u32x4_t*)(base + off);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 load16(const uint8_t* src, int need_lo, int need_hi) {
    const uintptr_t a = (uintptr_t)src & ~(uintptr_t)15;
    uint4 x = make_uint4(0, 0, 0, 0), y = x;
    if (a + 16 > (uintptr_t)(src + need_lo)) x = gload16(a);
    if (a + 16 < (uintptr_t)(src + need_hi)) y = gload16(a + 16);
    return window16(x, y, (uint32_t)((uintptr_t)src - a));
}

__device__ __forceinline__ uint32_t bytemask(int n) {   // low n bytes (n clamped to [0, 4])
    return n <= 0 ? 0u : (n >= 4 ? 0xffffffffu : (1u << (8 * n)) - 1u);
}

// shift a 16-byte window right by one byte
__device__ __forceinline__ void shr8(uint4& w) {
    w.x = __builtin_amdgcn_alignbyte(w.y, w.x, 1);
    w.y = __builtin_amdgcn_alignbyte(w.z, w.y, 1);
    w.z = __builtin_amdgcn_alignbyte(w.w, w.z, 1);
    w.w >>= 8;
}

// Iterate the bytes of text[lo, hi) in order: BODY sees `c` (the byte) and `i` (its index relative
// to lo).  One window load per 16 bytes, a runtime loop per byte (a wavefront leaves it as soon as
// its last lane is done, instead of stepping through whole predicated chunks).  (Loading each aligned
// chunk once with a one-ahead prefetch instead measured 20% slower in k_pair_eval: more VALU, and
// the prefetch of a run that ends early is wasted.)
#define PII_FOR_BYTES(text, lo, hi, ...)                                                         \
    for (int _j = (lo); _j < (hi); _j += 16) {                                                    \
        const int _n = (hi) - _j < 16 ? (hi) - _j : 16;                                           \
        uint4 _w = load16((text) + _j, 0, _n);                                                    \
        for (int _k = 0; _k < _n; ++_k) {                                                         \
            const uint32_t c = _w.x & 0xffu;                                                      \
            const int i = _j - (lo) + _k;                                                         \
            (void)i;                                                                              \
            __VA_ARGS__;                                                                          \
            shr8(_w);                                                                             \
        }                                                                                         \
    }

// ---------------------------------------------------------------------------------- validators
// SURVEY A.1 / B.4, one forward pass over the match's n bytes, read through a byte source: MemSrc
// (16-byte windows from memory) or RegSrc (the first 32 bytes, loaded once before the validator
// dispatch -- a wavefront's lanes run different validators one after another, and loads inside each
// would serialise one memory latency per validator kind).  src.each(n, f) calls f(byte, index).
struct MemSrc {
    const uint8_t* q;
    template <class F>
    __device__ __forceinline__ void each(int n, F&& f) const {
        PII_FOR_BYTES(q, 0, n, { f(c, i); })
    }
    __device__ __forceinline__ uint32_t word1() const { return load16(q, 4, 8).y; }    // bytes 4..7
};
struct RegSrc {
    uint4 a, b;                     // bytes [0, 16), [16, 32)
    template <class F>
    __device__ __forceinline__ void each(int n, F&& f) const {
        uint4 w = a;
        const int m = n < 16 ? n : 16;
        for (int k = 0; k < m; ++k) {
            f(w.x & 0xffu, k);
            shr8(w);
        }
        w = b;
        for (int k = 16; k < n; ++k) {
            f(w.x & 0xffu, k);
            shr8(w);
        }
    }
    __device__ __forceinline__ uint32_t word1() const { return a.y; }
};
// bytes [q, q + 32) as a register window (only the aligned chunks holding one of the n bytes are read)
__device__ __forceinline__ RegSrc load32(const uint8_t* q, int n) {
    const uintptr_t a0 = (uintptr_t)q & ~(uintptr_t)15;
    const uint32_t off = (uint32_t)((uintptr_t)q - a0);
    const uintptr_t end = (uintptr_t)q + (uintptr_t)n;
    uint4 c0 = gload16(a0), c1 = make_uint4(0, 0, 0, 0), c2 = c1;
    if (a0 + 16 < end) c1 = gload16(a0 + 16);
    if (a0 + 32 < end) c2 = gload16(a0 + 32);
    return RegSrc{window16(c0, c1, off), window16(c1, c2, off)};
}

template <class S>
__device__ inline bool v_luhn(const S src, int n) {
    // digit k (from the left) is doubled iff (cnt - 1 - k) is odd: keep both parities' sums
    int sa = 0, sb = 0, cnt = 0;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        if (is_digit(c)) {
            // (value selects, not branches assigning different variables: those make the compiler
            // pick the variable's address and keep it in scratch)
            const int d = (int)(c - '0');
            const int dd = d * 2 > 9 ? d * 2 - 9 : d * 2;
            const bool odd = cnt & 1;
            sa += odd ? dd : d;
            sb += odd ? d : dd;
            ++cnt;
        }
    });
    const int s = ((cnt - 1) & 1) ? sb : sa;
    return cnt >= 2 && s % 10 == 0;
}

template <class S>
__device__ inline bool v_nanp(const S src, int n) {
    int k = 0;
    bool ok = true;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        if (is_digit(c)) {
            if ((k == 0 || k == 3) && c < '2') ok = false;
            ++k;
        }
    });
    return ok && k == 10;
}

template <class S>
__device__ inline bool v_ssn(const S src, int n) {
    int k = 0;
    uint32_t area = 0, group = 0, serial = 0;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        if (is_digit(c)) {
            const uint32_t d = c - '0';
            area = k < 3 ? area * 10 + d : area;
            group = (k >= 3 && k < 5) ? group * 10 + d : group;
            serial = k >= 5 ? serial * 10 + d : serial;
            ++k;
        }
    });
    return k == 9 && area != 0 && area != 666 && area < 900 && group != 0 && serial != 0;
}

template <class S>
__device__ inline bool v_ein(const S src, int n) {
    int k = 0;
    uint32_t p = 0;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        if (is_digit(c)) {
            if (k < 2) p = p * 10 + (c - '0');
            ++k;
        }
    });
    if (k != 9) return false;
    const uint64_t lo = 0xfffdffffcff1fc7eull, hi = 0x0000000cfdff3f9full;   // oracle EIN_PREFIXES
    return p < 64 ? ((lo >> p) & 1) : ((hi >> (p - 64)) & 1);
}

template <class S>
__device__ inline bool v_ipv4(const S src, int n) {
    int parts = 0, len = 0;
    uint32_t val = 0;
    bool ok = true;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        const bool dot = c == '.', dig = is_digit(c);
        ok = ok && !(dot && (len == 0 || len > 3 || val > 255)) && (dot || dig);
        parts += dot ? 1 : 0;
        val = dot ? 0u : (dig ? val * 10 + (c - '0') : val);
        len = dot ? 0 : (dig ? len + 1 : len);
    });
    if (len == 0 || len > 3 || val > 255) ok = false;     // the final field
    return ok && parts + 1 == 4;
}

// ISO 3166-1 alpha-2, bit (a-'A')*26 + (b-'A')  (oracle ISO3166)
__constant__ const uint32_t ISO3166_BITS[22] = {0xeedf5978u, 0xdeddbdefu, 0x15843f27u, 0x0e00d480u, 0xb0095c00u, 0x0015fb9fu,
                              0x7818068du, 0x0340400fu, 0xf42b1d00u, 0xfd4f8141u, 0x25d7fffcu, 0x0100084bu,
                              0x538f3c40u, 0x40000001u, 0xfdf15100u, 0x9fbb3ae7u, 0x0410419au, 0x00408557u,
                              0x00004002u, 0x00100000u, 0x00400408u, 0x00000001u};

template <class S>
__device__ inline bool v_swift(const S src, int n) {
    if (n != 8 && n != 11) return false;
    const uint32_t w = src.word1();
    const uint32_t a = ((w >> 0) & 0xffu) - 'A', b = ((w >> 8) & 0xffu) - 'A';
    if (a >= 26u || b >= 26u) return false;
    const uint32_t i = a * 26 + b;
    return (ISO3166_BITS[i >> 5] >> (i & 31)) & 1;
}

// mod-97 of the string rotated by four characters (spaces skipped), in one forward pass:
// value(chars[4:]) * 10^digits(chars[0:4]) + value(chars[0:4])  (mod 97)
template <class S>
__device__ inline bool v_iban(const S src, int n) {
    int len = 0;
    uint32_t head = 0, headpow = 1, tail = 0;
    bool ok = true;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        if (c != ' ') {
            uint32_t v, m;
            if (is_digit(c)) {
                v = c - '0';
                m = 10;
            } else if (c - 'A' < 26u) {
                v = c - 55;
                m = 100;
            } else {
                ok = false;
                v = 0;
                m = 1;
            }
            // head / headpow take the first four characters (< 100^4 < 2^27: no reduction needed);
            // tail is reduced only when it could overflow (one modulo per few characters)
            const bool h4 = len < 4;
            head = h4 ? head * m + v : head;
            headpow = h4 ? headpow * m : headpow;
            uint32_t t = h4 ? tail : tail * m + v;
            if (t >= (1u << 24)) t %= 97;
            tail = t;
            ++len;
        }
    });
    if (!ok || len < 15 || len > 34) return false;
    return ((tail % 97) * (headpow % 97) + head % 97) % 97 == 1;
}

template <class S>
__device__ inline bool validate_src(int id, const S src, int n) {
    switch (id) {
        case 0: return true;
        case 1: return v_luhn(src, n);
        case 2: return v_nanp(src, n);
        case 3: return v_ssn(src, n);
        case 4: return v_ein(src, n);
        case 5: return v_ipv4(src, n);
        case 6: return v_swift(src, n);
        case 7: return v_iban(src, n);
        default: return false;
    }
}

// luhn / nanp / ssn / ein / ipv4 in ONE pass: a wavefront whose lanes hold different validators
// steps the match bytes once instead of once per validator kind (each kind's loop would run with the
// lanes of the other kinds idle).  Same results as v_luhn ... v_ipv4 (which the IBAN / SWIFT / long
// paths and the window kernels keep using).
template <class S>
__device__ inline bool v_digits(int id, const S src, int n) {
    int cnt = 0, sa = 0, sb = 0;                  // luhn
    uint32_t v9 = 0, d0 = 0, d3 = 0;              // the first nine digits as a number; digits 0 and 3
    int parts = 0, len = 0;                       // ipv4
    uint32_t val = 0;
    bool ok4 = true;
    src.each(n, [&](uint32_t c, int) __attribute__((always_inline)) {
        const bool dig = is_digit(c), dot = c == '.';
        const uint32_t d = dig ? c - '0' : 0u;
        const int dd = d * 2 > 9 ? (int)(d * 2 - 9) : (int)(d * 2);
        const bool odd = cnt & 1;
        sa += dig ? (odd ? dd : (int)d) : 0;
        sb += dig ? (odd ? (int)d : dd) : 0;
        v9 = (dig && cnt < 9) ? v9 * 10 + d : v9;
        d0 = (dig && cnt == 0) ? d : d0;
        d3 = (dig && cnt == 3) ? d : d3;
        cnt += dig ? 1 : 0;
        ok4 = ok4 && !(dot && (len == 0 || len > 3 || val > 255)) && (dot || dig);
        parts += dot ? 1 : 0;
        val = dot ? 0u : (dig ? val * 10 + d : val);
        len = dot ? 0 : (dig ? len + 1 : len);
    });
    switch (id) {
        case 1: return cnt >= 2 && (((cnt - 1) & 1) ? sb : sa) % 10 == 0;                  // luhn
        case 2: return cnt == 10 && d0 >= 2 && d3 >= 2;                                       // nanp
        case 3: {                                                                             // ssn
            const uint32_t area = v9 / 1000000u, group = (v9 / 10000u) % 100u, serial = v9 % 10000u;
            return cnt == 9 && area != 0 && area != 666 && area < 900 && group != 0 && serial != 0;
        }
        case 4: {                                                                             // ein
            if (cnt != 9) return false;
            const uint32_t p = v9 / 10000000u;
            const uint64_t lo = 0xfffdffffcff1fc7eull, hi = 0x0000000cfdff3f9full;   // oracle EIN_PREFIXES
            return p < 64 ? ((lo >> p) & 1) : ((hi >> (p - 64)) & 1);
        }
        case 5: return ok4 && !(len == 0 || len > 3 || val > 255) && parts + 1 == 4;        // ipv4
        default: return false;
    }
}

// matches of up to 32 bytes (every shipped validator's but a spaced IBAN's) are read once, up front
__device__ inline bool validate(int id, const uint8_t* q, int n) {
    if (id == 0) return true;
    if (n <= 32) {
        const RegSrc r = load32(q, n);
        return (id >= 1 && id <= 5) ? v_digits(id, r, n) : validate_src(id, r, n);
    }
    return validate_src(id, MemSrc{q}, n);
}

// ---------------------------------------------------------------------------------- DFA runners
// descriptor layout (compiler.put): tr_off, fl_off, cm_off, ncols, start_bot, start_w, start_n, n_states
// In the kernels' LDS images every transition entry is  next_state | flags(next_state) << 14
// (FIRST: bit 14 = a match ended before the byte just consumed, bit 15 = terminal; HOT: bit 14 =
// accept), so one step is two dependent LDS reads (byte class, transition).
constexpr uint32_t DFA_STATE_MASK = 0x3fffu;
struct Pool {
    const uint16_t* trans;
    const uint8_t* cmap;
};

// Anchored leftmost-first run of FIRST DFA `d` from byte s of text[0, L): the end `re` would report
// for a match starting at s, or -1 (compiler.build_first_dfa semantics).  Split in two so a caller
// can bound the lockstep cost: first_begin consumes at most one 16-byte window (the byte before s,
// which picks the start state, then up to 15 bytes) and either finishes or leaves a resumable
// {state, next position, last match end}; first_resume finishes it.
#ifndef FIRST_WINDOW
#define FIRST_WINDOW 16             // the byte before s + 15 steps (at most 16: one window load; 9 measured slower)
#endif
struct FirstState {
    uint32_t st;
    int pos;    // next byte to consume
    int last;   // end of the last match seen, -1 none
};

// byte K of a 16-byte window
template <int K>
__device__ __forceinline__ uint32_t wbyte(const uint4& w) {
    const uint32_t x = (K & 8) ? ((K & 4) ? w.w : w.z) : ((K & 4) ? w.y : w.x);
    return (x >> ((K & 3) * 8)) & 0xffu;
}
// byte classes of bytes H .. H + 7 of a window, issued together before the steps that use them (a
// class does not depend on the automaton state, so a step waits on one LDS read instead of two)
template <int H>
__device__ __forceinline__ void classes8(const uint8_t* cm, const uint4& w, uint32_t (&cl)[8]) {
    cl[0] = cm[wbyte<H + 0>(w)];
    cl[1] = cm[wbyte<H + 1>(w)];
    cl[2] = cm[wbyte<H + 2>(w)];
    cl[3] = cm[wbyte<H + 3>(w)];
    cl[4] = cm[wbyte<H + 4>(w)];
    cl[5] = cm[wbyte<H + 5>(w)];
    cl[6] = cm[wbyte<H + 6>(w)];
    cl[7] = cm[wbyte<H + 7>(w)];
}

// FIRST steps over the first n (<= 8) bytes whose classes are cl, byte 0 at text position p0:
// false = the run ended (r holds its result in `last`)
__device__ __forceinline__ bool first_steps8(const uint16_t* tr, uint32_t nc, const uint32_t (&cl)[8], int n,
                                             int p0, uint32_t& st, int& last) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (k < n) {
            const uint32_t e = tr[st * nc + cl[k]];
            st = e & DFA_STATE_MASK;
            if (e & 0x4000u) last = p0 + k;
            if (e & 0x8000u) return false;
        }
    }
    return true;
}

__device__ __forceinline__ int first_finish(const Pool& pool, const int32_t* d, const uint8_t* text, int L,
                                            FirstState& r) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* cm = pool.cmap + d[2];
    const uint32_t nc = (uint32_t)d[3];
    uint32_t st = r.st;
    int last = r.last;
    for (int j = r.pos; j < L; j += 16) {
        const int n = L - j < 16 ? L - j : 16;
        const uint4 w = load16(text + j, 0, n);
        uint32_t cl[8];
        classes8<0>(cm, w, cl);
        if (!first_steps8(tr, nc, cl, n, j, st, last)) return last;
        if (n > 8) {
            classes8<8>(cm, w, cl);
            if (!first_steps8(tr, nc, cl, n - 8, j + 8, st, last)) return last;
        }
    }
    if (tr[st * nc + nc - 1] & 0x4000u) last = L;
    return last;
}

// returns the run's result (>= -1) when finished inside the first window, or -2 with `r` saved
__device__ __forceinline__ int first_begin(const Pool& pool, const int32_t* d, const uint8_t* text, int s, int L,
                                           FirstState& r) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* cm = pool.cmap + d[2];
    const uint32_t nc = (uint32_t)d[3];
    const int lo = s == 0 ? 0 : s - 1;
    // lockstep window: most runs end within a few bytes (median 5 steps at config 2), so a
    // wavefront steps FIRST_WINDOW bytes in lockstep and the longer runs continue densely
    const int hi = L - lo < FIRST_WINDOW ? L : lo + FIRST_WINDOW;
    uint4 w = load16(text + lo, 0, hi - lo > 0 ? hi - lo : 1);
    uint32_t st;
    if (s == 0) {
        st = (uint32_t)d[4];
    } else {
        st = (uint32_t)(is_word(w.x & 0xffu) ? d[5] : d[6]);
        shr8(w);
    }
    int last = -1;
    const int n = hi - s;
    if (n > 0) {
        uint32_t cl[8];
        classes8<0>(cm, w, cl);
        if (!first_steps8(tr, nc, cl, n, s, st, last)) return last;
        if (n > 8) {
            classes8<8>(cm, w, cl);
            if (!first_steps8(tr, nc, cl, n - 8, s + 8, st, last)) return last;
        }
    }
    if (hi >= L) {
        if (tr[st * nc + nc - 1] & 0x4000u) last = L;
        return last;
    }
    r.st = st;
    r.pos = hi;
    r.last = last;
    return -2;
}

__device__ __forceinline__ int first_run(const Pool& pool, const int32_t* d, const uint8_t* text, int s, int L) {
    FirstState r;
    const int e = first_begin(pool, d, text, s, L, r);
    return e != -2 ? e : first_finish(pool, d, text, L, r);
}

// Unanchored HOT DFA over text[lo, hi) with the window edges as text edges (re.search semantics).
// Four bytes' classes are read together before their steps (a class does not depend on the state,
// so a step waits on one LDS read instead of two); a runtime loop over the 4-byte groups keeps the
// unrolled part (and k_pair_eval's registers) small.  hot_span steps text[lo, hi) from state st:
// true = an accept.
__device__ __forceinline__ bool hot_span(const uint16_t* tr, const uint8_t* cm, uint32_t nc, const uint8_t* text,
                                         int lo, int hi, uint32_t& st) {
    for (int j = lo; j < hi; j += 16) {
        const int n = hi - j < 16 ? hi - j : 16;
        uint4 w = load16(text + j, 0, n);
#pragma unroll 1
        for (int g = 0; g < n; g += 4) {
            const uint32_t x = w.x;
            const uint32_t c0 = cm[x & 0xffu], c1 = cm[(x >> 8) & 0xffu], c2 = cm[(x >> 16) & 0xffu], c3 = cm[x >> 24];
            const uint32_t cl[4] = {c0, c1, c2, c3};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (g + k < n) {
                    const uint32_t e = tr[st * nc + cl[k]];
                    if (e & 0x4000u) return true;
                    st = e & DFA_STATE_MASK;
                }
            }
            w = make_uint4(w.y, w.z, w.w, 0u);
        }
    }
    return false;
}

__device__ __forceinline__ bool hot_run(const Pool& pool, const int32_t* d, const uint8_t* text, int lo, int hi) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* cm = pool.cmap + d[2];
    const uint32_t nc = (uint32_t)d[3];
    uint32_t st = (uint32_t)d[4];
    if (hot_span(tr, cm, nc, text, lo, hi, st)) return true;
    return (tr[st * nc + nc - 1] & 0x4000u) != 0;
}

}  // namespace pii
