// pii_device.h - per-lane building blocks of the scan-and-redact pipeline (gfx950).
//
// Validators restate SURVEY.md Appendix A.1 / oracle/pii_oracle.py (v_luhn ... v_iban), the DFA
// runners execute the tables built by context-based-pii_amd/compiler.py.  Everything here is a
// plain __device__ function; the kernels in pii_engine.hip compose them.
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

// ---------------------------------------------------------------------------------- validators
// SURVEY A.1 / B.4.  q = matched bytes [0, n).
__device__ inline bool v_luhn(const uint8_t* q, int n) {
    int s = 0, cnt = 0;
    for (int i = n - 1; i >= 0; --i) {
        uint32_t c = q[i];
        if (!is_digit(c)) continue;
        int x = (int)(c - '0');
        if (cnt & 1) {
            x *= 2;
            if (x > 9) x -= 9;
        }
        s += x;
        ++cnt;
    }
    return cnt >= 2 && s % 10 == 0;
}

// digit-field validators accumulate the fields on the fly (no local arrays -> no scratch)
__device__ inline bool v_nanp(const uint8_t* q, int n) {
    int k = 0;
    bool ok = true;
    for (int i = 0; i < n; ++i) {
        const uint32_t c = q[i];
        if (!is_digit(c)) continue;
        if ((k == 0 || k == 3) && c < '2') ok = false;
        ++k;
    }
    return ok && k == 10;
}

__device__ inline bool v_ssn(const uint8_t* q, int n) {
    int k = 0;
    uint32_t area = 0, group = 0, serial = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t c = q[i];
        if (!is_digit(c)) continue;
        const uint32_t d = c - '0';
        if (k < 3) area = area * 10 + d;
        else if (k < 5) group = group * 10 + d;
        else serial = serial * 10 + d;
        ++k;
    }
    return k == 9 && area != 0 && area != 666 && area < 900 && group != 0 && serial != 0;
}

__device__ inline bool v_ein(const uint8_t* q, int n) {
    int k = 0;
    uint32_t p = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t c = q[i];
        if (!is_digit(c)) continue;
        if (k < 2) p = p * 10 + (c - '0');
        ++k;
    }
    if (k != 9) return false;
    const uint64_t lo = 0xfffdffffcff1fc7eull, hi = 0x0000000cfdff3f9full;   // oracle EIN_PREFIXES
    return p < 64 ? ((lo >> p) & 1) : ((hi >> (p - 64)) & 1);
}

__device__ inline bool v_ipv4(const uint8_t* q, int n) {
    int parts = 0, len = 0;
    uint32_t val = 0;
    for (int i = 0; i <= n; ++i) {
        uint32_t c = i < n ? q[i] : '.';
        if (c == '.') {
            if (len == 0 || len > 3 || val > 255) return false;
            ++parts;
            len = 0;
            val = 0;
        } else if (is_digit(c)) {
            val = val * 10 + (c - '0');
            ++len;
        } else {
            return false;
        }
    }
    return parts == 4;
}

// ISO 3166-1 alpha-2, bit (a-'A')*26 + (b-'A')  (oracle ISO3166)
__constant__ const uint32_t ISO3166_BITS[22] = {0xeedf5978u, 0xdeddbdefu, 0x15843f27u, 0x0e00d480u, 0xb0095c00u, 0x0015fb9fu,
                              0x7818068du, 0x0340400fu, 0xf42b1d00u, 0xfd4f8141u, 0x25d7fffcu, 0x0100084bu,
                              0x538f3c40u, 0x40000001u, 0xfdf15100u, 0x9fbb3ae7u, 0x0410419au, 0x00408557u,
                              0x00004002u, 0x00100000u, 0x00400408u, 0x00000001u};

__device__ inline bool v_swift(const uint8_t* q, int n) {
    const uint32_t* iso = ISO3166_BITS;
    if (n != 8 && n != 11) return false;
    uint32_t a = q[4] - 'A', b = q[5] - 'A';
    if (a >= 26u || b >= 26u) return false;
    uint32_t i = a * 26 + b;
    return (iso[i >> 5] >> (i & 31)) & 1;
}

__device__ inline bool v_iban(const uint8_t* q, int n) {
    int len = 0;
    for (int i = 0; i < n; ++i) len += q[i] != ' ';
    if (len < 15 || len > 34) return false;
    // rotate: chars 4.. then 0..3 (spaces skipped)
    uint32_t r = 0;
    for (int pass = 0; pass < 2; ++pass) {
        int k = 0;
        for (int i = 0; i < n; ++i) {
            uint32_t c = q[i];
            if (c == ' ') continue;
            bool take = pass == 0 ? k >= 4 : k < 4;
            ++k;
            if (!take) continue;
            if (is_digit(c)) r = (r * 10 + (c - '0')) % 97;
            else if (c - 'A' < 26u) r = (r * 100 + (c - 55)) % 97;
            else return false;
        }
    }
    return r == 1;
}

__device__ inline bool validate(int id, const uint8_t* q, int n) {
    switch (id) {
        case 0: return true;
        case 1: return v_luhn(q, n);
        case 2: return v_nanp(q, n);
        case 3: return v_ssn(q, n);
        case 4: return v_ein(q, n);
        case 5: return v_ipv4(q, n);
        case 6: return v_swift(q, n);
        case 7: return v_iban(q, n);
        default: return false;
    }
}

// ---------------------------------------------------------------------------------- DFA runners
// descriptor layout (compiler.put): tr_off, fl_off, cm_off, ncols, start_bot, start_w, start_n, n_states
struct Pool {
    const uint16_t* trans;
    const uint8_t* flags;
    const uint8_t* cmap;
};

template <int K>
__device__ __forceinline__ uint32_t chunk_byte(const uint4& w) {
    const uint32_t x = (K & 8) ? ((K & 4) ? w.w : w.z) : ((K & 4) ? w.y : w.x);
    return (x >> ((K & 3) * 8)) & 0xffu;
}

// Text access for the DFA runners: aligned 16-byte chunks (one chunk prefetched ahead) with
// compile-time byte extraction, instead of one dependent byte load per DFA step.  A chunk is only
// loaded when it contains at least one byte of the requested range; an aligned 16-byte block never
// straddles a page, so reading all of it is safe.
#define PII_DFA_STREAM(BODY)                                                                      \
    {                                                                                             \
        const uint8_t* pa = text + lo;                                                            \
        const uint4* cp = reinterpret_cast<const uint4*>((uintptr_t)pa & ~(uintptr_t)15);         \
        int j = lo - (int)((uintptr_t)pa & 15);   /* position of byte 0 of chunk *cp */           \
        uint4 w = *cp;                                                                            \
        uint4 wn = j + 16 < hi ? cp[1] : w;                                                       \
        for (;;) {                                                                                \
            const uint4 cur = w;                                                                  \
            w = wn;                                                                               \
            if (j + 32 < hi) wn = cp[2];                                                          \
            BODY(0) BODY(1) BODY(2) BODY(3) BODY(4) BODY(5) BODY(6) BODY(7)                       \
            BODY(8) BODY(9) BODY(10) BODY(11) BODY(12) BODY(13) BODY(14) BODY(15)                 \
            j += 16;                                                                              \
            ++cp;                                                                                 \
            if (j >= hi) break;                                                                   \
        }                                                                                         \
    }

// Anchored leftmost-first run of FIRST DFA `d` from byte s of text[0, L): returns the end `re`
// would report for a match starting at s, or -1.  (compiler.build_first_dfa: flags bit0 = a match
// ended before the char just consumed, bit1 = terminal.)
__device__ __forceinline__ int first_run(const Pool& pool, const int32_t* d, const uint8_t* text, int s, int L) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* fl = pool.flags + d[1];
    const uint8_t* cm = pool.cmap + d[2];
    const int nc = d[3];
    int st = s == 0 ? d[4] : (is_word(text[s - 1]) ? d[5] : d[6]);
    int last = -1;
    if (s < L) {
        const int lo = s, hi = L;
#define PII_FIRST_STEP(K)                                                                         \
        if (j + (K) >= lo && j + (K) < hi) {                                                      \
            st = tr[st * nc + cm[chunk_byte<K>(cur)]];                                            \
            const uint32_t f = fl[st];                                                            \
            if (f & 1) last = j + (K);                                                            \
            if (f & 2) return last;                                                               \
        }
        PII_DFA_STREAM(PII_FIRST_STEP)
#undef PII_FIRST_STEP
    }
    st = tr[st * nc + nc - 1];
    if (fl[st] & 1) last = L;
    return last;
}

// Unanchored HOT DFA over text[lo, hi) with the window edges as text edges (re.search semantics)
__device__ __forceinline__ bool hot_run(const Pool& pool, const int32_t* d, const uint8_t* text, int lo, int hi) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* fl = pool.flags + d[1];
    const uint8_t* cm = pool.cmap + d[2];
    const int nc = d[3];
    int st = d[4];
    if (lo < hi) {
#define PII_HOT_STEP(K)                                                                           \
        if (j + (K) >= lo && j + (K) < hi) {                                                      \
            st = tr[st * nc + cm[chunk_byte<K>(cur)]];                                            \
            if (fl[st]) return true;                                                              \
        }
        PII_DFA_STREAM(PII_HOT_STEP)
#undef PII_HOT_STEP
    }
    st = tr[st * nc + nc - 1];
    return fl[st] != 0;
}

}  // namespace pii
