// pii_engine.hip - MI355X (gfx950) scan-and-redact engine: kernels + C ABI (include/pii_engine.h).
//
// Replaces the remote de-identification call of the reference,
//   main_service/main.py:728  dlp_client.deidentify_content(request)   (inside call_dlp_for_redaction,
//   main.py:580-773), and the Redis context record main.py:366-374 / 403.
//
// Pipeline per batch (one HIP stream, no host round trip until pii_sync):
//   k_chunk_index  lane -> utterance ranges of ~BYTES_PER_LANE bytes (load balance, no halo needed);
//                  per-row defaults
//   k_lane_bits    utterance-start words per lane and 64-byte block (lane-interleaved, coalesced)
//   k_halo         start states of the lanes a long row's slice boundaries cut (one workgroup per row)
//   k_scan         REVERSE two-automaton DFA scan, tables in LDS.  D = relaxed detector prefilter,
//                  K = exact context keywords.  Emits candidate STARTS (events) per lane
//   k_pairs        agent-row context group (extract_expected_pii, main.py:558-578); (start, pattern)
//                  pair queue
//   k_ctx_scan / k_ctx_apply   per-conversation context (Redis SETEX/GET + TTL) as a segmented scan
//   k_pair_first   leftmost-first confirmation of every pair (FIRST DFAs in LDS)
//   k_pair_eval    validators + hotword windows (HOT DFAs in LDS) under the row's context variant
//   k_select       finditer skipping, exclusion, overlap resolution, output sizing
//   k_scan_*       exclusive scans -> output byte offsets and span offsets
//   k_finalize     capacity / error check (device side)
//   k_redact       prefix-sum scatter of kept bytes and "[INFO_TYPE]" tokens, span list, histogram
//   k_ctx_commit   write the per-conversation context back (only when the call succeeded)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pii_engine.h"
#include "pii_device.h"

using namespace pii;

namespace {

constexpr int NE_MAX = 2;          // excluder patterns
#ifndef SCAN_INLINE_HALO
#define SCAN_INLINE_HALO 1          // k_scan steps a cut lane's halo itself (no k_halo launch per SCAN group)
#endif
constexpr size_t SCAN_LDS_TWO_WG = 80 * 1024;   // k_scan tables up to this: two workgroups per CU
#ifndef SCAN1_BLOCK
#define SCAN1_BLOCK 768
#endif
#ifndef SCAN1_WAVES
#define SCAN1_WAVES 6
#endif
constexpr int SCAN_BLOCK = SCAN1_BLOCK;          // 12 waves: two workgroups (<= 80 KiB of tables each) fill the 6 waves/SIMD the VGPRs allow
constexpr int CTX_BLOCK = 1024;            // (context aggregates are allocated per CTX_BLOCK rows)
constexpr int SCAN_ITEMS = 8;      // items per thread in the offset scans (blocked, 16-byte accesses)
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;
#ifndef BYTES_PER_LANE_N
#define BYTES_PER_LANE_N 1024
#endif
constexpr uint32_t BYTES_PER_LANE = BYTES_PER_LANE_N;    // largest scan lane (big batches)
constexpr uint32_t MIN_LANE_SHIFT = 7;        // smallest scan lane, 128 B (small batches need lanes, not bytes)
constexpr int KW_NONE = 0x7fff;
constexpr int PAIRS_UCAP = 1024;   // utterances a wavefront stages in LDS (k_pairs_flat)

enum : uint32_t { ERR_CAPACITY = 1, ERR_ORDER = 2, ERR_SLOT = 4, ERR_QUEUE = 8, ERR_RING = 16, ERR_STITCH = 32,
                  ERR_ARGS = 64, ERR_EXT = 128 };
// a call whose declared batch size was wrong (ERR_ARGS) or whose queues overflowed (ERR_QUEUE, re-run by
// pii_sync) stops every later stage
constexpr uint32_t ERR_ABORT = ERR_QUEUE | ERR_ARGS;

struct Event {
    uint32_t pos;   // candidate start, relative to the batch base
    uint16_t sd;    // D transition index (row + class) that reported it
    uint16_t sk;    // K transition index (row + class)
};

struct RulesDev {
    int P, G, T, V, SD, CD, d_start, SK, CK, k_start, n_hot, min_len;
    int kw_always_min, NE;
    int CDs, CKs;                // row strides of the SCAN tables (CD / CK rounded up to even; a WIDE
                                 // group's D: to a multiple of 4)
    int dsh;                     // D entry = row byte offset >> dsh (| flags): 0, or 1 for a WIDE SCAN
                                 // group >= 1 (D table up to 128 KiB; its class words carry no K half)
    uint32_t n_dacc, n_kacc;     // D / K accept sets
    const uint32_t* cmap4;    // [256] 2*classD | 2*classK << 16 (byte offsets)
    const uint16_t* td;       // [SD*CDs] LDS byte address of the next row in k_scan | accept (bit 0)
                              //   | the next row's end-of-text transition accepts (bit 1)
    const uint16_t* tk;       // [SK*CKs]
    const uint16_t* d_accid;  // [SD*CDs]
    const uint32_t* d_acc_off;
    const uint16_t* d_acc_ids;
    const uint16_t* k_accid;  // [SK*CKs]
    const uint16_t* k_acc_min;  // per K accept set: smallest context group
    const uint16_t* d_npair;    // [SD*CDs] per D transition: pairs of its accept set (k_pairs count pass)
    const uint16_t* k_grp;      // [SK*CKs] per K transition: smallest context group it accepts, or KW_NONE
    const uint16_t* det_type;
    const uint8_t* det_val;
    const uint8_t* det_lik;
    const uint8_t* det_exidx;   // excluder slot or 0xff
    const int32_t* first_desc;  // [P*8]
    const int32_t* hot_rule;    // [n_hot*4] wb, wa, fixed, rel
    const int32_t* hot_desc;    // [n_hot*8]
    const uint8_t* var_enabled;  // [V*T]
    const uint8_t* var_minlik;   // [V]
    const uint32_t* rule_off;    // [V*T+1]
    const uint16_t* rule_ids;
    const uint32_t* excl_off;    // [V*T+1]
    const uint16_t* excl_ids;
    const uint32_t* tok_off;     // [T+1] into tok_bytes: "[NAME]"
    const uint8_t* tok_bytes;
    uint32_t nl_off;             // tok_bytes[nl_off] = '\n' (the re-scan window separator)
};

// ------------------------------------------------------------------------------- lane geometry
// A scan LANE is the set of utterances whose START lies in one slice [c << sh, (c+1) << sh) of the
// batch, sliced in the ADDRESS space (positions are shifted by r0 = batch base address & 63, so a
// slice boundary is a 64-byte boundary of the text buffer).  A LONG row (longer than long_min bytes:
// a whole transcript, a realtime join, a joined re-scan window) is in addition CUT at every slice
// boundary strictly inside it, so it is spread over many lanes instead of running on one thread:
// the lane holding its start ends at the first cut, every further slice is a lane of its own.
// Lanes are scanned with a halo (k_scan) and stitched by verification (k_scan_fix, k_sel_*).
struct Geo {
    const uint64_t* offs;
    const uint32_t* first_utt;
    const uint4* lanes;     // per lane {lo, hi, u0 | clo << 31, u1 | chi << 31} (k_lane_count); null before
    uint64_t base;          // offs[0]
    uint32_t n_utt, n_chunks, sh, r0, long_min;
};
struct Lane {
    uint32_t lo, hi;        // byte range [lo, hi), batch relative
    uint32_t u0, u1;        // utterances [u0, u1) overlapping it
    bool clo, chi;          // cut at lo (continues a long row) / at hi (the long row goes on)
};
constexpr uint32_t NO_CUTS = 0xffffffffu;     // long_min that disables cutting (window re-scan)
constexpr uint32_t SCAN_HALO = 128;            // bytes a lane scans past a cut before it emits

__device__ __forceinline__ int64_t g_off(const Geo& g, uint32_t u) { return (int64_t)(g.offs[u] - g.base); }
__device__ __forceinline__ int64_t g_cpos(const Geo& g, uint32_t k) { return ((int64_t)k << g.sh) - (int64_t)g.r0; }

// slice boundary k (1 <= k < n_chunks) cuts the row first_utt[k] - 1 (the last row starting before it)
__device__ __forceinline__ bool g_cut(const Geo& g, uint32_t k) {
    if (k == 0 || k >= g.n_chunks || g.long_min == NO_CUTS) return false;
    const uint32_t f = g.first_utt[k];
    if (f == 0) return false;
    const int64_t p = g_cpos(g, k), s = g_off(g, f - 1), e = g_off(g, f);
    return p > s && p < e && (e - s) > (int64_t)g.long_min;
}

__device__ __forceinline__ Lane g_lane_slow(const Geo& g, uint32_t c) {
    Lane L;
    const uint32_t f0 = g.first_utt[c], f1 = g.first_utt[c + 1];
    L.clo = g_cut(g, c);
    L.chi = g_cut(g, c + 1);
    L.lo = (uint32_t)(L.clo ? g_cpos(g, c) : g_off(g, f0));
    L.hi = (uint32_t)(L.chi ? g_cpos(g, c + 1) : g_off(g, f1));
    L.u0 = L.clo ? f0 - 1 : f0;
    L.u1 = f1;
    return L;
}

// (rows are < 2^31: the host bounds bytes + 2 * rows below 2^32)
__device__ __forceinline__ uint4 lane_pack(const Lane& L) {
    return make_uint4(L.lo, L.hi, L.u0 | (L.clo ? 0x80000000u : 0u), L.u1 | (L.chi ? 0x80000000u : 0u));
}
__device__ __forceinline__ Lane g_lane(const Geo& g, uint32_t c) {
    if (!g.lanes) return g_lane_slow(g, c);
    const uint4 x = g.lanes[c];
    Lane L;
    L.lo = x.x;
    L.hi = x.y;
    L.u0 = x.z & 0x7fffffffu;
    L.u1 = x.w & 0x7fffffffu;
    L.clo = (x.z >> 31) != 0;
    L.chi = (x.w >> 31) != 0;
    return L;
}

// the lane's event arena starts here (capacity >= its emitted positions + utterance starts, see
// k_scan); its findings arena at fd + lo / min_len + c
__device__ __forceinline__ uint64_t ev_base(const Lane& L, uint32_t c) {
    return (uint64_t)L.lo + c + L.u0 + (L.clo ? 1u : 0u);
}

// the lanes of cut row r: ca holds its start, (ca, kb] continue it
__device__ __forceinline__ void row_lanes(const Geo& g, uint32_t r, uint32_t& ca, uint32_t& kb, int64_t& s_r,
                                          int64_t& e_r) {
    s_r = g_off(g, r);
    e_r = g_off(g, r + 1);
    ca = (uint32_t)((s_r + g.r0) >> g.sh);                                         // lane holding the start
    kb = (uint32_t)min<int64_t>((int64_t)g.n_chunks - 1, (e_r + g.r0 - 1) >> g.sh);   // last continuation
}

// first_utt[c] = first utterance starting at or after slice c (c in [0, n_chunks]); also writes every
// row's defaults (no findings: out_len = len; keyword group = the always-present group for AGENT rows,
// else -1) with coalesced stores, and lists the rows that will be cut (long rows).
constexpr int CI_ROWS = 4;          // rows per thread in k_chunk_index (16-byte row-default stores)
static_assert(CI_ROWS == 4, "k_chunk_index stores the row defaults as one uint4 / int4");
// a row [s, e) (batch relative) that some slice boundary cuts (the test of g_cut)
__device__ __forceinline__ bool cut_row(uint64_t s, uint64_t e, uint32_t r0, uint32_t lane_shift, uint32_t n_chunks,
                                        uint32_t long_min) {
    if (long_min == NO_CUTS || e - s <= long_min) return false;
    const uint64_t kk = ((s + r0) >> lane_shift) + 1;                 // first boundary after its start
    return kk < n_chunks && ((int64_t)(kk << lane_shift) - (int64_t)r0) < (int64_t)e;
}

// first_utt over the slices a cut row r spans, (slice of its start, slice of its end]: row r + 1
__device__ __forceinline__ void fill_after(uint32_t* __restrict__ first_utt, uint32_t r, uint64_t s, uint64_t e,
                                           uint32_t n_utt, uint32_t n_chunks, uint32_t lane_shift, uint32_t r0,
                                           uint32_t t0, uint32_t step) {
    const uint64_t c_lo = ((s + r0) >> lane_shift) + 1;
    uint64_t c_hi = (r + 1 == n_utt) ? n_chunks : (e + r0) >> lane_shift;
    if (c_hi > n_chunks) c_hi = n_chunks;
    for (uint64_t c = c_lo + t0; c <= c_hi; c += step) first_utt[c] = r + 1;
}

__global__ __launch_bounds__(256) void k_chunk_index(const uint64_t* __restrict__ offs, const uint8_t* __restrict__ role,
                                                     uint32_t n_utt, uint32_t n_chunks, uint32_t lane_shift, uint32_t r0,
                                                     uint32_t long_min, int kw_always,
                                                     uint32_t* __restrict__ first_utt, uint32_t* __restrict__ out_len,
                                                     int32_t* __restrict__ kw, uint32_t* __restrict__ wc_n,
                                                     uint32_t* __restrict__ long_rows, uint32_t* __restrict__ long_count,
                                                     uint32_t long_cap, uint64_t decl_base, uint64_t decl_bytes,
                                                     uint32_t* __restrict__ err) {
    const uint32_t u0 = (blockIdx.x * blockDim.x + threadIdx.x) * CI_ROWS;
    if (u0 > n_utt) return;
    const uint64_t base = offs[0];
    // the caller declared offsets[0] and the batch size (no host round trip): every later kernel sized
    // its work from them, so a wrong declaration stops the call
    if (u0 + CI_ROWS > n_utt && (base != decl_base || offs[n_utt] - base != decl_bytes)) atomicOr(err, (uint32_t)ERR_ARGS);
    // offsets of rows u0 - 1 .. u0 + CI_ROWS, issued together
    uint64_t o[CI_ROWS + 2];
#pragma unroll
    for (int k = 0; k < CI_ROWS + 2; ++k) {
        const int64_t u = (int64_t)u0 - 1 + k;
        o[k] = (u >= 0 && u <= (int64_t)n_utt) ? offs[u] : 0;
    }
    uint32_t ol[CI_ROWS];
    int32_t kv[CI_ROWS];
#pragma unroll
    for (int k = 0; k < CI_ROWS; ++k) {
        const uint32_t u = u0 + k;
        if (u > n_utt) break;
        // the slices after a CUT row are filled by k_fill_long, a workgroup per row (one thread storing a
        // 1 MB row's 1024 entries serialised this kernel); the rest here
        if (u == 0 || o[k + 1] - o[k] <= long_min ||
            !cut_row(o[k] - base, o[k + 1] - base, r0, lane_shift, n_chunks, long_min)) {
            const uint64_t c_lo = u > 0 ? ((o[k] - base + r0) >> lane_shift) + 1 : 0;
            uint64_t c_hi = (u == n_utt) ? n_chunks : (o[k + 1] - base + r0) >> lane_shift;
            if (c_hi > n_chunks) c_hi = n_chunks;
            for (uint64_t c = c_lo; c <= c_hi; ++c) first_utt[c] = u;
        }
        ol[k] = 0;
        kv[k] = -1;
        if (u < n_utt) {
            const uint64_t len = o[k + 2] - o[k + 1];
            ol[k] = (uint32_t)len;
            kv[k] = (role[u] == PII_ROLE_AGENT && kw_always != KW_NONE) ? kw_always : -1;
            if (wc_n) wc_n[u] = 0;
            const bool cut = len > long_min && cut_row(o[k + 1] - base, o[k + 2] - base, r0, lane_shift, n_chunks, long_min);
            // one counter atomic per wavefront (a window step cuts ~1k short rows: one atomic per row
            // serialised on the counter, 7 -> 20 us)
            const uint64_t bal = __ballot(cut);
            uint32_t wbase = 0;
            const int lane = threadIdx.x & 63, lead = bal ? __builtin_ctzll(bal) : 0;
            if (bal && lane == lead) wbase = atomicAdd(long_count, (uint32_t)__popcll(bal));
            wbase = __shfl(wbase, lead);
            if (cut) {
                const uint32_t at = wbase + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
                if (at < long_cap) {
                    long_rows[at] = u;
                } else {
                    atomicOr(err, (uint32_t)ERR_STITCH);      // (sized by ensure_scratch: internal)
                    fill_after(first_utt, u, o[k + 1] - base, o[k + 2] - base, n_utt, n_chunks, lane_shift, r0, 0, 1);
                }
            }
        }
    }
    // row defaults (no findings: out_len = len; keyword group = the always-present group for AGENT
    // rows, else -1): 16-byte stores for a full group (the arrays are the engine's, 16-byte aligned)
    if (u0 + CI_ROWS <= n_utt) {
        *reinterpret_cast<uint4*>(out_len + u0) = make_uint4(ol[0], ol[1], ol[2], ol[3]);
        *reinterpret_cast<int4*>(kw + u0) = make_int4(kv[0], kv[1], kv[2], kv[3]);
    } else {
        for (int k = 0; k < CI_ROWS && u0 + k < n_utt; ++k) {
            out_len[u0 + k] = ol[k];
            kw[u0 + k] = kv[k];
        }
    }
}

// first_utt over the slices of the listed cut rows (k_chunk_index left them), one workgroup per row
__global__ __launch_bounds__(256) void k_fill_long(const uint64_t* __restrict__ offs, uint32_t n_utt,
                                                   uint32_t n_chunks, uint32_t lane_shift, uint32_t r0,
                                                   const uint32_t* __restrict__ long_rows,
                                                   const uint32_t* __restrict__ long_count, uint32_t long_cap,
                                                   uint32_t* __restrict__ first_utt) {
    const uint32_t nrows = min(*long_count, long_cap);
    const uint64_t base = offs[0];
    for (uint32_t ri = blockIdx.x; ri < nrows; ri += gridDim.x) {
        const uint32_t r = long_rows[ri];
        fill_after(first_utt, r, offs[r] - base, offs[r + 1] - base, n_utt, n_chunks, lane_shift, r0, threadIdx.x,
                   blockDim.x);
    }
}

// ------------------------------------------------------------------------------------- k_scan
// Each lane owns the utterances whose START falls in its BYTES_PER_LANE slice of the batch, i.e. one
// contiguous byte range [lo, hi], and walks it right to left in aligned 64-byte blocks (the next
// block is prefetched while the current one is stepped).  Per 16 bytes the byte-class lookups are
// issued first (independent of the automaton state), then the two automata take 16 dependent steps.
// Utterance boundaries are crossed in-stream: reaching an utterance's first byte applies the
// end-of-text pseudo class (the "start of text" of the reverse automata) and resets the state.
// A step does no range test: the bytes of the edge blocks outside [lo, hi] are stepped too (the
// boundary bit at hi + 1 -- a virtual one at the batch end -- resets the state before byte hi), and
// only an event (rare) is range-checked.  A transition with bit 15 set appends {pos, D transition,
// K transition} to the lane's event region; nothing is written per utterance (k_chunk_index wrote
// the defaults).  Table entries are BYTE offsets (row * classes * 2) so one add forms an LDS address.
template <int K>
__device__ __forceinline__ uint32_t byte_c(const uint4& w) {
    const uint32_t x = (K & 8) ? ((K & 4) ? w.w : w.z) : ((K & 4) ? w.y : w.x);
    return (x >> ((K & 3) * 8)) & 0xffu;
}

// Utterance-start words, lane-interleaved: word[i * n_lanes + t] holds, for the lane in scan slot t,
// its i-th block from the top (address-aligned 64-byte block b_top - i, b = (position + r0) >> 6):
// bit k <=> a non-empty utterance of the lane starts at position 64b - r0 + k, or that position is
// the lane's scan TOP (the position after its last scanned byte: the next lane's first start, the
// batch end, or the end of a cut lane's halo), which resets the automata before the lane's last
// byte.  All lanes of a wavefront read word i at the same iteration, so the scan's word loads are
// coalesced.  Blocks past LANE_WORDS use a slow path.
constexpr int LANE_WORDS = 32;

// exclusive end of the bytes lane L scans (a lane cut at hi starts from the state its halo produced,
// k_halo, instead of stepping the halo itself)
__device__ __forceinline__ uint32_t scan_top(const Geo& g, const Lane& L) { return L.hi; }

// bits of lane c's i-th block from the top (the slow path for i >= LANE_WORDS: binary search over the
// lane's utterances; everything is re-derived from (c, i) so the scan keeps nothing live for it)
__device__ __attribute__((noinline)) uint64_t block_bits_slow(const Geo g, uint32_t c, uint32_t i) {
    const Lane L = g_lane(g, c);
    const uint32_t top = scan_top(g, L);
    const int64_t blk = (((int64_t)top - 1 + g.r0) >> 6) - i;
    const int64_t plo = blk * 64 - g.r0, phi = plo + 64;       // positions [plo, phi)
    uint64_t bits = 0;
    if (!L.chi && (int64_t)top >= plo && (int64_t)top < phi) bits |= 1ull << (top - plo);
    const uint32_t vmin = L.u0 + (L.clo ? 1u : 0u);
    if (vmin >= L.u1) return bits;
    // largest v in [vmin, u1) with start < phi
    uint32_t a = vmin, b = L.u1 - 1;
    if (g_off(g, a) >= phi) return bits;
    while (a < b) {
        const uint32_t m = (a + b + 1) >> 1;
        if (g_off(g, m) < phi) a = m;
        else b = m - 1;
    }
    for (int64_t v = a; v >= (int64_t)vmin; --v) {
        const int64_t sv = g_off(g, (uint32_t)v);
        if (sv < plo) break;
        if (g_off(g, (uint32_t)v + 1) > sv) bits |= 1ull << (sv - plo);
    }
    return bits;
}

// ------------------------------------------------------------------ lane order (k_scan balance)
// A wavefront of k_scan runs as long as its longest lane (a lane is ~1 KiB of WHOLE utterances, so
// lengths spread over ~0.5-2 KiB: in batch order a wavefront's lanes are only ~80% busy).  The scan
// therefore takes its lanes in order of decreasing length: a counting sort on 32-byte length buckets
// gives slot -> lane (lane_perm) and lane -> slot (lane_pos); k_lane_bits writes each lane's start
// words at its slot, so the scan's word loads stay coalesced.  The order is not deterministic (block
// reservations race) but only the thread mapping depends on it: every lane's events, counts and
// arena are the same.
constexpr int LANE_NB = 128;                       // length buckets: 0 = longest (>= 127*32 B)
__device__ __forceinline__ uint32_t lane_bucket(const Geo& g, uint32_t c) {
    const Lane L = g_lane(g, c);
    const uint32_t len = scan_top(g, L) - min(L.lo, scan_top(g, L));
    return (uint32_t)(LANE_NB - 1) - min<uint32_t>(len >> 5, LANE_NB - 1);
}

constexpr uint32_t LANE_SORT_CHUNK = 1024;         // lanes per workgroup (4 per thread; ~1k workgroups at config 2)

// k_scan2's lane split (see k_scan2 below for the design)
static_assert(BYTES_PER_LANE == 1024, "k_scan2's word rows are sized for 1 KiB lanes");
constexpr int HB_A = (3 * BYTES_PER_LANE) / 32 + 2;   // word rows of chain A: its half-blocks from its top
constexpr int HB_B = 32;      // word rows of chain B (from its top, byte s - 1), stored after A's

// The split of a lane for k_scan2: a non-empty utterance start s in (lo, top), not 32-byte aligned (so
// A's last half-block holds byte s - 1), that makes the longer chain shortest; only lanes no cut
// touches (their events and arena are the plain ones).  Returns (s - lo) | capA << 16 (capA: the arena
// entries A may fill -- positions [s, hi - 1], one accept each, + the end-of-text events of its
// starts), 0 = no split; kmax = half-blocks of the longer chain (the lane's k_scan2 iterations).
template <class Off>
__device__ __forceinline__ uint32_t choose_split(const Lane& L, uint32_t top, uint32_t r0, Off uoff, uint32_t& kmax) {
    const int64_t hb_hi = ((int64_t)top - 1 + r0) >> 5, hb_lo = ((int64_t)L.lo + r0) >> 5;
    int64_t best = hb_hi - hb_lo + 1, vs = -1, s = 0;
    if (!L.clo && !L.chi && L.u0 + 1 < L.u1) {
        int64_t sv = uoff(L.u0 + 1);
        for (int64_t v = (int64_t)L.u0 + 1; v < (int64_t)L.u1; ++v) {
            if (sv >= (int64_t)top) break;
            const int64_t sn = uoff(v + 1);
            if (sv > (int64_t)L.lo && ((sv + r0) & 31) != 0 && sn != sv) {
                const int64_t hs = (sv + r0) >> 5;
                const int64_t na = hb_hi - hs + 1, nb = hs - hb_lo + 1, mx = max(na, nb);
                if (na <= HB_A && nb <= HB_B && mx < best) {
                    best = mx;
                    vs = v;
                    s = sv;
                }
            }
            sv = sn;
        }
    }
    kmax = (uint32_t)best;
    if (vs < 0) return 0;
    const int64_t cap = ((int64_t)top - s) + ((int64_t)L.u1 - vs);
    if (s - (int64_t)L.lo >= 65536 || cap >= 65536) {
        kmax = (uint32_t)(hb_hi - hb_lo + 1);
        return 0;
    }
    return (uint32_t)(s - L.lo) | (uint32_t)cap << 16;
}

// the longer chain's half-blocks of lane L with split sp (the k_scan2 lane order's key)
__device__ __forceinline__ uint32_t split_kmax(const Lane& L, uint32_t top, uint32_t r0, uint32_t sp) {
    const uint32_t hb_hi = (top - 1 + r0) >> 5, hb_lo = (L.lo + r0) >> 5;
    if (!sp) return hb_hi - hb_lo + 1;
    const uint32_t hs = (L.lo + (sp & 0xffffu) + r0) >> 5;
    return max(hb_hi - hs + 1, hs - hb_lo + 1);
}

// also records every lane's geometry (g.lanes is null here; later kernels read the records); SPLIT
// (k_scan2): also each lane's split (spl), and the lanes are ordered by the longer chain's length
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_lane_count(const Geo g, uint32_t* __restrict__ bucket_cnt,
                                                    uint4* __restrict__ lanes, uint32_t* __restrict__ spl) {
    __shared__ uint32_t h[LANE_NB];
    for (int i = threadIdx.x; i < LANE_NB; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint32_t c0 = blockIdx.x * LANE_SORT_CHUNK, c1 = min(c0 + LANE_SORT_CHUNK, g.n_chunks);
    for (uint32_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
        const Lane L = g_lane_slow(g, c);
        lanes[c] = lane_pack(L);
        const uint32_t len = L.hi - min(L.lo, L.hi);
        uint32_t key = len >> 5;
        if constexpr (SPLIT) {
            uint32_t km = 0;
            spl[c] = len ? choose_split(L, L.hi, g.r0, [&](int64_t u) { return g_off(g, (uint32_t)u); }, km) : 0u;
            key = len ? km : 0u;
        }
        const uint32_t bk = (uint32_t)(LANE_NB - 1) - min(key, (uint32_t)(LANE_NB - 1));
        atomicAdd(&h[bk], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < LANE_NB; i += blockDim.x)
        if (h[i]) atomicAdd(&bucket_cnt[i], h[i]);
}

// bucket_cnt[0..NB) = counts (k_lane_count), bucket_cnt[NB..2NB) = reservation cursors (zeroed)
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_lane_place(const Geo g, uint32_t* __restrict__ bucket_cnt,
                                                    uint32_t* __restrict__ lane_perm, uint32_t* __restrict__ lane_pos,
                                                    const uint32_t* __restrict__ spl) {
    constexpr int PER = LANE_SORT_CHUNK / 256;
    __shared__ uint32_t base[LANE_NB], h[LANE_NB];
    if (threadIdx.x < 64) {                        // exclusive prefix of the counts, one wavefront
        uint32_t run = 0;
        for (int k = 0; k < LANE_NB; k += 64) {
            const uint32_t v = bucket_cnt[k + threadIdx.x];
            uint32_t incl = v;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(incl, d);
                if ((int)threadIdx.x >= d) incl += o;
            }
            base[k + threadIdx.x] = run + incl - v;
            run += __shfl(incl, 63);
        }
    }
    for (int i = threadIdx.x; i < LANE_NB; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint32_t c0 = blockIdx.x * LANE_SORT_CHUNK;
    uint32_t bk[PER], rk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t c = c0 + j * 256 + threadIdx.x;
        bk[j] = 0;
        if (c < g.n_chunks) {
            if constexpr (SPLIT) {
                const Lane L = g_lane(g, c);
                const uint32_t key = L.hi > L.lo ? split_kmax(L, L.hi, g.r0, spl[c]) : 0u;
                bk[j] = (uint32_t)(LANE_NB - 1) - min(key, (uint32_t)(LANE_NB - 1));
            } else {
                bk[j] = lane_bucket(g, c);
            }
        }
        rk[j] = c < g.n_chunks ? atomicAdd(&h[bk[j]], 1u) : 0u;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < LANE_NB; i += blockDim.x)
        if (h[i]) base[i] += atomicAdd(&bucket_cnt[LANE_NB + i], h[i]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t c = c0 + j * 256 + threadIdx.x;
        if (c < g.n_chunks) {
            const uint32_t t = base[bk[j]] + rk[j];
            lane_perm[t] = c;
            lane_pos[c] = t;
        }
    }
}

// table entries are absolute LDS byte addresses of the next row, bit 0 = accept (scan_tables); k_scan
// has no static LDS, so its dynamic region starts at LDS address 0 and an entry IS the address
constexpr uint32_t SCAN_TD_BASE = 1024;     // after the 256-entry class map
constexpr uint32_t SCAN_SPREAD_BYTES = 512; // k_scan's 256 group masks (scan_spread), after the K table
typedef const __attribute__((address_space(3))) uint16_t lds_u16_t;
__device__ __forceinline__ uint32_t lds_u16(uint32_t addr) {
    return *reinterpret_cast<lds_u16_t*>((size_t)addr);
}

// the state a lane carries across a cut: both automata's current rows (flag bits masked off)
__device__ __forceinline__ uint32_t scan_state(uint32_t nd, uint32_t nk) { return (nd & 0xfffcu) | ((nk & 0xfffcu) << 16); }

// The state a lane cut at hi starts from: both automata stepped right to left over the SCAN_HALO
// bytes after the cut (clamped to the row) from the start state, with the tables in LDS in k_scan's
// layout (k_halo stages them); k_scan_fix verifies the result against the neighbour's real state.
// The halo is read as aligned 16-byte chunks (each holds a batch byte, as k_scan's reads do), the
// bytes taken from registers: per-byte loads from 64 lanes' distant rows thrashed L2.
__device__ uint32_t halo_state(const RulesDev& R, const Geo& g, const uint8_t* __restrict__ text, const Lane& L) {
    const uint32_t top = (uint32_t)min<int64_t>((int64_t)L.hi + SCAN_HALO, g_off(g, L.u1));
    const uint32_t tk_base = SCAN_TD_BASE + (uint32_t)(R.SD * R.CDs / 2) * 4;
    const uintptr_t tb = (uintptr_t)(text + g.base);
    uint32_t nd = 0, nk = 0, pm = 0xffffffffu;
    if (top <= L.hi) return scan_state(nd, nk);
    const uintptr_t a_hi = (tb + top - 1) & ~(uintptr_t)15, a_lo = (tb + L.hi) & ~(uintptr_t)15;
    uint4 nx = gload16(a_hi);
    for (uintptr_t a = a_hi;; a -= 16) {
        const uint4 w = nx;
        if (a > a_lo) nx = gload16(a - 16);                // the next chunk's load runs under these steps
        const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 15; j >= 0; --j) {
            const uintptr_t b = a + (uintptr_t)j;
            if (b >= tb + L.hi && b < tb + top) {
                const uint32_t x = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
                    (size_t)(4u * ((wd[j >> 2] >> (8 * (j & 3))) & 0xffu)));
                const uint32_t ad = ((nd & ~pm & 0xfffcu) << R.dsh) + (x & 0xffffu);
                const uint32_t ak = (nk & ~pm & 0xfffcu) + (R.SK > 1 ? (x >> 16) : tk_base);   // (groups >= 1: K stub)
                nd = lds_u16(ad);
                nk = lds_u16(ak);
                pm = 0;
            }
        }
        if (a == a_lo) break;
    }
    return scan_state(nd, nk);
}

// Halo states of every cut lane, one workgroup per long row (the k_scan_fix grid), the group's scan
// tables staged in LDS: the lanes (ca, kb] continue long row r, so lanes [ca, kb) are cut at hi.
// Only long rows have cut lanes, so a batch without them costs one early exit.
constexpr int HALO_BLOCK = 1024;    // k_halo: lanes of a long row in flight per workgroup (one per CU)
__global__ __launch_bounds__(HALO_BLOCK) void k_halo(const RulesDev R, const Geo g, const uint8_t* __restrict__ text,
                                              const uint32_t* __restrict__ long_rows,
                                              const uint32_t* __restrict__ long_count,
                                              uint32_t* __restrict__ lane_st, const uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
    const uint32_t nrows = *long_count;
    if (blockIdx.x >= nrows || (*err & (ERR_ARGS | ERR_STITCH))) return;
    {
        const int nd_words = R.SD * R.CDs / 2, nk_words = R.SK * R.CKs / 2;
        const uint32_t* g_td = reinterpret_cast<const uint32_t*>(R.td);
        const uint32_t* g_tk = reinterpret_cast<const uint32_t*>(R.tk);
        uint32_t* d_td = smem32 + SCAN_TD_BASE / 4;
        uint32_t* d_tk = d_td + nd_words;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) smem32[i] = R.cmap4[i];
        for (int i = threadIdx.x; i < nd_words; i += blockDim.x) d_td[i] = g_td[i];
        for (int i = threadIdx.x; i < nk_words; i += blockDim.x) d_tk[i] = g_tk[i];
    }
    __syncthreads();
    for (uint32_t ri = blockIdx.x; ri < nrows; ri += gridDim.x) {
        uint32_t ca, kb;
        int64_t s_r, e_r;
        row_lanes(g, long_rows[ri], ca, kb, s_r, e_r);
        for (uint32_t c = ca + threadIdx.x; c < kb; c += blockDim.x) {
            const Lane L = g_lane(g, c);
            if (L.chi && scan_top(g, L) > L.lo) lane_st[2 * c] = halo_state(R, g, text, L);
        }
    }
}

// The utterance offsets of a wavefront's 64 lanes, staged in LDS as 16-bit offsets from the start of
// the wavefront's first slice: the rows that START in its slices (at most 64 << sh <= 64 KiB past
// it); the row before them (a cut row) and the row after them are kept in registers.  Config 5's
// 57-byte rows are ~1150 per wavefront: 32-bit offsets in the same 16 KiB of LDS held 1024, and
// k_lane_bits fell back to global loads (183 -> 80 us at config 5).  (k_pairs_flat staged this way
// measured slower, 213 -> 327 us: its binary searches pay for the range tests; it keeps 32 bits.)
constexpr int WROWS_CAP = 2048;
static_assert(BYTES_PER_LANE * 64 <= 65536, "16-bit offsets within a wavefront's slices");
struct WaveRows {
    uint16_t* so;
    int64_t lo;            // relative position of the wavefront's first slice
    uint32_t uf, ue;       // rows starting in the wavefront's slices: [uf, ue)
    int64_t o_prev, o_end; // offsets of rows uf - 1 and ue
    bool staged;
    __device__ __forceinline__ void stage(const Geo& g, uint32_t cw0, uint32_t cw1, int lane, uint16_t* buf) {
        so = buf;
        uf = g.first_utt[cw0];
        ue = g.first_utt[cw1];
        lo = g_cpos(g, cw0);
        staged = ue - uf <= (uint32_t)WROWS_CAP;
        o_prev = uf > 0 ? g_off(g, uf - 1) : 0;
        o_end = g_off(g, ue);
        if (staged)
            for (uint32_t k = lane; k < ue - uf; k += 64) so[k] = (uint16_t)(g_off(g, uf + k) - lo);
    }
    __device__ __forceinline__ int64_t off(const Geo& g, uint32_t u) const {
        if (u == ue) return o_end;
        if (staged && u >= uf && u < ue) return lo + so[u - uf];
        if (u + 1 == uf) return o_prev;
        return g_off(g, u);
    }
};

// one thread per lane; the wavefront stages its utterance offsets in LDS first (coalesced loads)
__global__ __launch_bounds__(256) void k_lane_bits(const Geo g, const uint32_t* __restrict__ lane_pos,
                                                   uint64_t* __restrict__ words) {
    // (16 KiB of LDS per workgroup leaves the kernel at its register occupancy, 7 waves/SIMD)
    __shared__ uint16_t s_off[4][WROWS_CAP];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t cw0 = c - lane;
    const uint32_t cw1 = min(cw0 + 64, g.n_chunks);
    WaveRows W;
    if (cw0 < g.n_chunks) W.stage(g, cw0, cw1, lane, s_off[wv]);
    __syncthreads();
    if (c >= g.n_chunks) return;
    auto uoff = [&](int64_t u) { return W.off(g, (uint32_t)u); };
    const Lane L = g_lane(g, c);
    const uint32_t top = scan_top(g, L);
    if (top <= L.lo) return;
    const int64_t b_hi = ((int64_t)top - 1 + g.r0) >> 6, b_lo = ((int64_t)L.lo + g.r0) >> 6;
    const int64_t nw = min<int64_t>(b_hi - b_lo + 1, LANE_WORDS);
    const uint32_t slot = lane_pos[c];
    const int64_t vmin = (int64_t)L.u0 + (L.clo ? 1 : 0);
    int64_t v = (int64_t)L.u1 - 1;
    int64_t sv = v >= vmin ? uoff(v) : 0;
    for (int64_t i = 0; i < nw; ++i) {
        const int64_t plo = (b_hi - i) * 64 - g.r0;
        uint64_t bits = 0;
        if (i == 0 && !L.chi && (int64_t)top >= plo && (int64_t)top < plo + 64) bits |= 1ull << (top - plo);
        while (v >= vmin && sv >= plo) {
            if (sv < plo + 64 && uoff(v + 1) > sv) bits |= 1ull << (sv - plo);
            --v;
            if (v >= vmin) sv = uoff(v);
        }
        words[(uint64_t)i * g.n_chunks + slot] = bits;
    }
}

// the lane's events go to its own arena (ev + ab, ab = ev_base, 32-bit: the host bounds bytes + rows
// + lanes of a batch below 2^32): only positions in its emission range [lo_r, lo_r + len_r] are recorded
__device__ __forceinline__ void scan_emit(Event* __restrict__ ev, uint32_t ab, uint32_t& cnt, uint32_t pos,
                                          uint32_t lo_r, uint32_t len_r, uint32_t ad, uint32_t ak, uint32_t tk_base) {
    if (pos - lo_r <= len_r) {
        Event e;
        e.pos = (uint32_t)pos;
        e.sd = (uint16_t)((ad - SCAN_TD_BASE) >> 1);     // transition index (row * CD + class)
        e.sk = (uint16_t)((ak - tk_base) >> 1);
        // (the index is formed here, opaque to the optimiser: a hoisted 64-bit ev + ab per lane would
        // hold two VGPRs across the scan loop -- and spill there)
        uint32_t idx = ab + cnt++;
        asm volatile("" : "+v"(idx));
        ev[idx] = e;
    }
}

// the group mask for utterance-start bits sb (bit j: byte j starts one): every accept bit (even bits),
// and the end-of-text bit 2 (7 - j) + 1 of each starting byte j (the m layout of SCAN_STEP8)
__device__ __forceinline__ uint32_t scan_spread(uint32_t sb) {
    uint32_t v = 0x5555u;
    for (int j = 0; j < 8; ++j)
        if (sb >> j & 1u) v |= 1u << (2 * (7 - j) + 1);
    return v;
}

// class word of byte K of a 16-byte chunk: the class map sits at LDS address 0, so the address is
// byte * 4 -- one SDWA shift of the byte lane of its dword
template <int K>
__device__ __forceinline__ uint32_t class_of(const uint4& w) {
    const uint32_t x = (K & 8) ? ((K & 4) ? w.w : w.z) : ((K & 4) ? w.y : w.x);
    uint32_t a;
    if constexpr ((K & 3) == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
            : "=v"(a) : "v"(x));
    else if constexpr ((K & 3) == 1)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
            : "=v"(a) : "v"(x));
    else if constexpr ((K & 3) == 2)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
            : "=v"(a) : "v"(x));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
            : "=v"(a) : "v"(x));
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>((size_t)a);
}

// byte classes of 8 bytes (HALF = 0: bytes 8..15 of the chunk, 1: bytes 0..7), issued together
#define SCAN_CLASSES8(W, H)                                                                       \
    cc[0] = class_of<(H) + 0>(W);                                                                 \
    cc[1] = class_of<(H) + 1>(W);                                                                 \
    cc[2] = class_of<(H) + 2>(W);                                                                 \
    cc[3] = class_of<(H) + 3>(W);                                                                 \
    cc[4] = class_of<(H) + 4>(W);                                                                 \
    cc[5] = class_of<(H) + 5>(W);                                                                 \
    cc[6] = class_of<(H) + 6>(W);                                                                 \
    cc[7] = class_of<(H) + 7>(W);

// v[j] for a per-lane j in 0..7 (a select tree: the arrays stay in registers)
__device__ __forceinline__ uint32_t sel8(const uint32_t (&v)[8], uint32_t j) {
    const bool b0 = j & 1u, b1 = j & 2u, b2 = j & 4u;
    const uint32_t v01 = b0 ? v[1] : v[0], v23 = b0 ? v[3] : v[2];
    const uint32_t v45 = b0 ? v[5] : v[4], v67 = b0 ? v[7] : v[6];
    const uint32_t v03 = b1 ? v23 : v01, v47 = b1 ? v67 : v45;
    return b2 ? v47 : v03;
}

// The events of one 8-byte group, in the order the per-step scan produced them (byte 7 first; on a
// byte, its accept before the end-of-text accept of an utterance start).  m holds 2 flag bits per
// byte j at bit 2 (7 - j): bit 0 = an automaton accepted on the byte (record its transitions ad[j],
// ak[j], start pos + 1), bit 1 = the byte starts an utterance and the destination row accepts at
// end of text (record the destination rows' EOT transitions, start pos).
__device__ __forceinline__ void scan_emit8(Event* __restrict__ ev, uint32_t ab, uint32_t& cnt, uint32_t m,
                                           const uint32_t (&ad)[8], const uint32_t (&ak)[8], uint32_t p0,
                                           uint32_t lo_r, uint32_t len_r, uint32_t tk_base, uint32_t eot_d,
                                           uint32_t eot_k, uint32_t dsh) {
    do {
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        const uint32_t j = 7u - (b >> 1);
        uint32_t a = sel8(ad, j), k = sel8(ak, j);
        uint32_t pos = p0 + j + 1u;
        if (b & 1u) {
            a = ((lds_u16(a) & 0xfffcu) << dsh) + eot_d;
            k = (lds_u16(k) & 0xfffcu) + eot_k;
            pos -= 1u;
        }
        scan_emit(ev, ab, cnt, pos, lo_r, len_r, a, k, tk_base);
    } while (m);
}

// One byte of both reverse automata.  nd/nk are the raw entries of the previous step: the destination
// row's offset from the START row (relayout puts the start state first) | flags.  pm is all ones iff
// the previous byte started an utterance, and then the row becomes the start row without a branch:
// (entry & ~pm & ~3) + class, the class word carrying the table bases (both halves stay below 64 KiB,
// so nothing carries between them).  The two dependent ALU ops between LDS reads are the whole
// per-byte chain.  Both flag bits of every byte are shifted into the top of m (one alignbit: byte j
// ends at bits 16 + 2 (7 - j)); the group's spread mask (LDS, indexed by its utterance-start bits)
// then keeps an end-of-text accept only on a byte that starts an utterance.
#define SCAN_STEP8(J, H)                                                                          \
    {                                                                                             \
        ad[J] = HK ? (nd & ~pm & 0xfffcu) + (cc[J] & 0xffffu) : ((nd & ~pm & 0xfffcu) << dsh) + cc[J];  \
        ak[J] = HK ? (nk & ~pm & 0xfffcu) + (cc[J] >> 16) : tk_base;                              \
        nd = lds_u16(ad[J]);                                                                      \
        if (HK) nk = lds_u16(ak[J]);                                                              \
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(pm) : "v"(b16), "n"((H) + (J)));                   \
        m = __builtin_amdgcn_alignbit(HK ? nd | nk : nd, m, 2);                                   \
    }

#define SCAN_GROUP8(W, H, OFF)                                                                    \
    {                                                                                             \
        uint32_t cc[8], ad[8], ak[8], m = 0;                                                      \
        SCAN_CLASSES8(W, H)                                                                       \
        const uint32_t mk = lds_u16(spread + 2u * ((b16 >> (H)) & 0xffu));                        \
        SCAN_STEP8(7, H) SCAN_STEP8(6, H) SCAN_STEP8(5, H) SCAN_STEP8(4, H)                       \
        SCAN_STEP8(3, H) SCAN_STEP8(2, H) SCAN_STEP8(1, H) SCAN_STEP8(0, H)                       \
        m = (m >> 16) & mk;                                                                       \
        if (__builtin_expect(m != 0, 0))                                                          \
            scan_emit8(ev, ab, cnt, m, ad, ak, bpos + (OFF) + (H), lo_r, len_r, tk_base, eot_d, eot_k, dsh); \
    }

#define SCAN_SUB(W, OFF)                                                                          \
    {                                                                                             \
        const uint32_t b16 = (uint32_t)(bits >> (OFF)) & 0xffffu;                                 \
        SCAN_GROUP8(W, 8, OFF)                                                                    \
        SCAN_GROUP8(W, 0, OFF)                                                                    \
    }


// Emission range of lane L: event positions [e_lo, e_hi].  A position is reported by the step over the
// byte before it, so a lane cut at lo leaves position lo to its left neighbour, and a lane cut at hi
// reports position hi itself (the right neighbour never steps byte hi - 1).
__device__ __forceinline__ void emit_range(const Lane& L, uint32_t& e_lo, uint32_t& e_len) {
    e_lo = L.lo + (L.clo ? 1u : 0u);
    const uint32_t e_hi = L.chi ? L.hi : L.hi - 1u;
    e_len = e_hi - e_lo;                 // wraps for an empty range: nothing is emitted
}

// HK = false: a SCAN group >= 1, whose K is the never-accepting one-row stub -- K is not stepped (its
// row stays the start row, its transition is the stub's class-0 entry), one LDS read less per byte
// NT: 768 threads (two workgroups per CU with tables <= 80 KiB, 6 waves / SIMD), or SCAN_BLOCK_WIDE for
// a WIDE group's table (one workgroup per CU: 16 waves instead of 12).  (256-thread workgroups for the
// window re-scan's small steps, to reach every CU instead of 123: 67 -> 73 us, not kept)
constexpr int SCAN_BLOCK_WIDE = 1024;
#ifndef SCAN_ABLATE
#define SCAN_ABLATE 0               // measurement builds only: 1 = k_scan returns after its table load
#endif
template <bool HK, int NT = SCAN_BLOCK>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == SCAN_BLOCK ? SCAN1_WAVES : 4, NT == SCAN_BLOCK ? SCAN1_WAVES : 4))) void k_scan(const RulesDev R, const Geo g, const uint8_t* __restrict__ text,
                                                     const uint64_t* __restrict__ words,
                                                     const uint32_t* __restrict__ lane_perm, Event* __restrict__ ev,
                                                     uint32_t* __restrict__ lane_cnt, uint32_t* __restrict__ lane_st,
                                                     const uint32_t* __restrict__ err, uint32_t ilv) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
    if (*err & ERR_ARGS) return;              // the declared batch size was wrong: nothing is sized for it
    // LDS: class map at 0 (256 x class words: D base + 2 classD | (K base + 2 classK) << 16), D table,
    // K table, group masks
    const int nd_words = R.SD * R.CDs / 2;      // rows padded to an even class count
    const int nk_words = R.SK * R.CKs / 2;
    const uint32_t tk_base = SCAN_TD_BASE + (uint32_t)nd_words * 4;
    {
        const uint32_t* g_td = reinterpret_cast<const uint32_t*>(R.td);
        const uint32_t* g_tk = reinterpret_cast<const uint32_t*>(R.tk);
        uint32_t* d_td = smem32 + SCAN_TD_BASE / 4;
        uint32_t* d_tk = d_td + nd_words;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) smem32[i] = R.cmap4[i];
        for (int i = threadIdx.x; i < nd_words; i += blockDim.x) d_td[i] = g_td[i];
        for (int i = threadIdx.x; i < nk_words; i += blockDim.x) d_tk[i] = g_tk[i];
        uint32_t* d_sp = d_tk + nk_words;
        for (int i = threadIdx.x; i < 128; i += blockDim.x) d_sp[i] = scan_spread(2 * i) | scan_spread(2 * i + 1) << 16;
    }
    __syncthreads();
    // slot (lanes longest first).  ilv (a grid of at most one workgroup per CU): the wavefronts are
    // dealt round-robin over the workgroups, so the longest lanes run one wavefront per CU instead of
    // sharing the first CU's LDS
    const uint32_t t = ilv ? ((threadIdx.x >> 6) * gridDim.x + blockIdx.x) * 64u + (threadIdx.x & 63u)
                           : blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= g.n_chunks) return;
#if SCAN_ABLATE == 1
    if (g.n_chunks != 0xffffffffu) return;      // (measurement: the table load only)
#endif
    const uint32_t c = lane_perm[t];
    const Lane L = g_lane(g, c);
    // positions relative to the batch base fit 32 bits (PII_MAX_BATCH_BYTES); 32-bit arithmetic keeps
    // the lane's bookkeeping small (VGPRs decide this kernel's occupancy)
    const uint32_t top = scan_top(g, L);
    const uint32_t end_r = (uint32_t)g_off(g, g.n_utt);
    uint32_t cnt = 0;
    if (top > L.lo) {
        uint32_t lo_r, len_r;
        emit_range(L, lo_r, len_r);
        const uint32_t ab = (uint32_t)ev_base(L, c);
        const uint32_t eot_d = SCAN_TD_BASE + 2u * (uint32_t)(R.CD - 1), eot_k = tk_base + 2u * (uint32_t)(R.CK - 1);
        const uint32_t spread = tk_base + (uint32_t)nk_words * 4;     // scan_spread table (after K)
        const uint32_t dsh = HK ? 0u : (uint32_t)R.dsh;               // (group 0 is never wide)
        // "previous byte started an utterance": start rows; a lane cut at hi continues from its halo state
        uint32_t nd = 0, nk = 0, pm = 0xffffffffu;
        if (L.chi) {
#if SCAN_INLINE_HALO
            // the lane's start state: its halo stepped here, from the tables already in LDS (a cut
            // lane is rare except in long rows, where every lane pays 128 of its 1024 steps); the
            // guess is kept for k_scan_fix, which checks it against the neighbour's real end state
            const uint32_t hs = halo_state(R, g, text, L);
            lane_st[2 * c] = hs;
#else
            const uint32_t hs = lane_st[2 * c];
#endif
            nd = hs & 0xffffu;
            nk = hs >> 16;
            pm = 0;
        }
        // aligned 64-byte blocks of the ADDRESS space, numbered from the one holding the batch base:
        // block bb covers relative positions [64 bb - r0, 64 bb - r0 + 64)
        const uint32_t r0 = g.r0;
        const uintptr_t tpb = (uintptr_t)(text + g.base) - r0;      // global loads (see gload16)
        const uint32_t bb_hi = (top - 1 + r0) >> 6, bb_lo = (L.lo + r0) >> 6;
        // the top block: only chunks holding a batch byte are read (the rest step as zero bytes
        // before the end-of-batch / next-utterance reset)
        const uint32_t q_end = (end_r - 1 + r0) >> 4;               // last chunk with a batch byte
        uint4 n0 = gload16(tpb + (uintptr_t)bb_hi * 64u), n1 = make_uint4(0, 0, 0, 0), n2 = n1, n3 = n1;
        if (4 * bb_hi + 1 <= q_end) n1 = gload16(tpb + (uintptr_t)bb_hi * 64u + 16);
        if (4 * bb_hi + 2 <= q_end) n2 = gload16(tpb + (uintptr_t)bb_hi * 64u + 32);
        if (4 * bb_hi + 3 <= q_end) n3 = gload16(tpb + (uintptr_t)bb_hi * 64u + 48);
        uint64_t nb = words[t];
        for (uint32_t bb = bb_hi;; --bb) {
            const uint4 w0 = n0, w1 = n1, w2 = n2, w3 = n3;
            const uint64_t bits = nb;
            if (bb > bb_lo) {
                const uintptr_t q = tpb + (uintptr_t)(bb - 1) * 64u;
                n0 = gload16(q);
                n1 = gload16(q + 16);
                n2 = gload16(q + 32);
                n3 = gload16(q + 48);
                const uint32_t i = bb_hi - (bb - 1);
                nb = i < (uint32_t)LANE_WORDS ? words[(uint64_t)i * g.n_chunks + t] : block_bits_slow(g, c, i);
            }
            const uint32_t bpos = 64u * bb - r0;        // relative position of the block's byte 0 (mod 2^32)
            SCAN_SUB(w3, 48)
            SCAN_SUB(w2, 32)
            SCAN_SUB(w1, 16)
            SCAN_SUB(w0, 0)
            if (bb == bb_lo) break;
        }
        if (L.clo) lane_st[2 * c + 1] = scan_state(nd, nk);        // lo is block aligned: state after byte lo
    }
    lane_cnt[c] = cnt;
}

// ------------------------------------------------------------------ k_scan2: two chains per lane
// k_scan is bound by one dependent LDS read per byte per lane (the D row of byte j is the entry read
// at byte j + 1): at the 6 waves/SIMD its VGPRs allow, 4.7 achieved, the CU's LDS idles between a
// wave's dependent reads (issue-active 24%, parked 39%).  k_scan2 gives each lane TWO independent
// chains.  k_lane_bits2 SPLITS a lane at one of its own utterance starts s near its middle: chain A
// steps [s, top) exactly as k_scan steps a lane [s, top), chain B steps [lo, s) from the start state --
// which is the single chain's state after it steps byte s (an utterance start resets both automata),
// so the split needs no halo and no verification, and the events are exactly the single chain's.
// The chains step interleaved, byte for byte, over 32-byte half-blocks (a block of text per chain
// in flight, as k_scan).  A keeps the events at positions >= s, B those < s (a position is reported
// by the step over the byte before it: A's last half-block holds byte s - 1, as s is not 32-byte
// aligned).  A writes into the lane's arena, B behind A's capacity; B's events are moved down behind
// A's at the end, so the arena holds the single chain's events in its order and no consumer changes.
// A lane without a usable utterance start (a cut lane, one long utterance) runs chain A alone.
// Register budget (80 VGPRs: 6 waves/SIMD in 768-thread workgroups, two per CU): per byte and chain
// one history word (both automata's rows, masked, packed; the emission re-derives the byte's class
// from the text) instead of k_scan's ad / ak, and per chain two 16-byte chunks of text, ping-pong: the
// next chunk is loaded as soon as the one in its registers has been stepped (no register copies, which
// would wait for the loads they copy), 16 bytes per chain = 32 interleaved steps ahead of its use.
// Word rows: k_scan2 runs for 1 KiB lanes with rows longer than 2 KiB cut (long_min), so a lane is
// shorter than 3 KiB and A's half-blocks always fit HB_A rows -- the loop needs no slow path, and its
// prefetch is branch-free (a finished chain re-reads its last half-block), so the compiler's counted
// vmcnt waits stay a whole half-block behind the loads.
// split[slot] = the lane's split (spl, by lane: k_lane_count); words32 rows [0, HB_A) = A's
// half-blocks from the lane's top, rows [HB_A, HB_A + HB_B) = B's from byte s - 1
__global__ __launch_bounds__(256) void k_lane_bits2(const Geo g, const uint32_t* __restrict__ lane_pos,
                                                    const uint32_t* __restrict__ spl, uint32_t* __restrict__ words,
                                                    uint32_t* __restrict__ split) {
    __shared__ uint16_t s_off[4][WROWS_CAP];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t cw0 = c - lane;
    const uint32_t cw1 = min(cw0 + 64, g.n_chunks);
    WaveRows W;
    if (cw0 < g.n_chunks) W.stage(g, cw0, cw1, lane, s_off[wv]);
    __syncthreads();
    if (c >= g.n_chunks) return;
    auto uoff = [&](int64_t u) { return W.off(g, (uint32_t)u); };
    const Lane L = g_lane(g, c);
    const uint32_t top = scan_top(g, L);
    if (top <= L.lo) return;                 // (k_scan2 reads nothing of an empty lane)
    const uint32_t slot = lane_pos[c];
    const uint64_t n = g.n_chunks;
    const int64_t r0 = g.r0;
    const int64_t vmin = (int64_t)L.u0 + (L.clo ? 1 : 0);
    const int64_t hb_hi = ((int64_t)top - 1 + r0) >> 5, hb_lo = ((int64_t)L.lo + r0) >> 5;
    const uint32_t sp = spl[c];
    split[slot] = sp;
    auto rows = [&](int64_t h0, int64_t nw, int64_t v, uint64_t row0, bool with_top) {
        int64_t sv = v >= vmin ? uoff(v) : 0;
        for (int64_t i = 0; i < nw; ++i) {
            const int64_t plo = (h0 - i) * 32 - r0;
            uint32_t bits = 0;
            if (with_top && i == 0 && (int64_t)top >= plo && (int64_t)top < plo + 32) bits |= 1u << (top - plo);
            while (v >= vmin && sv >= plo) {
                if (sv < plo + 32 && uoff(v + 1) > sv) bits |= 1u << (sv - plo);
                --v;
                if (v >= vmin) sv = uoff(v);
            }
            words[(row0 + (uint64_t)i) * n + slot] = bits;
        }
    };
    if (!sp) {
        rows(hb_hi, min<int64_t>(hb_hi - hb_lo + 1, HB_A), (int64_t)L.u1 - 1, 0, !L.chi);
        return;
    }
    // the utterance starting at s: the last one starting at or before it (a binary search of its rows)
    const int64_t s = (int64_t)L.lo + (sp & 0xffffu);
    int64_t a = vmin, b = (int64_t)L.u1 - 1;
    while (a < b) {
        const int64_t m = (a + b + 1) >> 1;
        if (uoff(m) <= s) a = m;
        else b = m - 1;
    }
    const int64_t hs = (s + r0) >> 5;
    rows(hb_hi, hb_hi - hs + 1, (int64_t)L.u1 - 1, 0, !L.chi);
    rows(hs, hs - hb_lo + 1, a, HB_A, false);
}

// the events of one chain's 8-byte group (scan_emit8's order); h[j] = the masked rows byte j was
// stepped from (HK: D | K << 16, the class re-derived from the group's text dwords; else the D address)
template <bool HK>
__device__ __forceinline__ void scan2_emit8(Event* __restrict__ ev, uint32_t ab, uint32_t& cnt, uint32_t m,
                                            const uint32_t (&h)[8], uint32_t w_lo, uint32_t w_hi, uint32_t p0,
                                            uint32_t lo_r, uint32_t len_r, uint32_t tk_base, uint32_t eot_d,
                                            uint32_t eot_k, uint32_t dsh) {
    do {
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        const uint32_t j = 7u - (b >> 1);
        const uint32_t hj = sel8(h, j);
        uint32_t a, k;
        if (HK) {
            const uint32_t by = (((j & 4u) ? w_hi : w_lo) >> (8u * (j & 3u))) & 0xffu;
            const uint32_t cw = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>((size_t)(4u * by));
            a = (hj & 0xffffu) + (cw & 0xffffu);
            k = (hj >> 16) + (cw >> 16);
        } else {
            a = hj;
            k = tk_base;
        }
        uint32_t pos = p0 + j + 1u;
        if (b & 1u) {
            a = ((lds_u16(a) & 0xfffcu) << dsh) + eot_d;
            k = (lds_u16(k) & 0xfffcu) + eot_k;
            pos -= 1u;
        }
        scan_emit(ev, ab, cnt, pos, lo_r, len_r, a, k, tk_base);
    } while (m);
}

// one byte of chain X (J: byte of the group, BIT: its bit in the half-block word)
#define S2_STEP1(X, J, BIT)                                                                       \
    {                                                                                             \
        if (HK) {                                                                                 \
            h##X[J] = ((nk##X << 16) | nd##X) & ~pm##X & 0xfffcfffcu;                             \
            uint32_t ad_, ak_;                                                                    \
            asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0" \
                : "=v"(ad_) : "v"(h##X[J]), "v"(c##X[J]));                                       \
            asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1" \
                : "=v"(ak_) : "v"(h##X[J]), "v"(c##X[J]));                                       \
            nd##X = lds_u16(ad_);                                                                 \
            nk##X = lds_u16(ak_);                                                                 \
            m##X = __builtin_amdgcn_alignbit(nd##X | nk##X, m##X, 2);                             \
        } else {                                                                                  \
            h##X[J] = ((nd##X & ~pm##X & 0xfffcu) << dsh) + c##X[J];                              \
            nd##X = lds_u16(h##X[J]);                                                             \
            m##X = __builtin_amdgcn_alignbit(nd##X, m##X, 2);                                     \
        }                                                                                         \
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(pm##X) : "v"(b##X), "n"(BIT));                      \
    }

#define S2_CLASSES8(C, W, H)                                                                      \
    C[0] = class_of<(H) + 0>(W);                                                                  \
    C[1] = class_of<(H) + 1>(W);                                                                  \
    C[2] = class_of<(H) + 2>(W);                                                                  \
    C[3] = class_of<(H) + 3>(W);                                                                  \
    C[4] = class_of<(H) + 4>(W);                                                                  \
    C[5] = class_of<(H) + 5>(W);                                                                  \
    C[6] = class_of<(H) + 6>(W);                                                                  \
    C[7] = class_of<(H) + 7>(W);

#define S2_STEP2(J, BIT) S2_STEP1(A, J, BIT) S2_STEP1(B, J, BIT)

// one 8-byte group of both chains: bytes H..H+7 of chunk WA / WB, at bit OFF + H of the words
#define S2_GROUP(WA, WB, H, OFF)                                                                  \
    {                                                                                             \
        uint32_t cA[8], cB[8], hA[8], hB[8], mA = 0, mB = 0;                                      \
        S2_CLASSES8(cA, WA, H)                                                                    \
        S2_CLASSES8(cB, WB, H)                                                                    \
        const uint32_t mkA = aliveA ? lds_u16(spread + 2u * ((bA >> ((OFF) + (H))) & 0xffu)) : 0u; \
        const uint32_t mkB = aliveB ? lds_u16(spread + 2u * ((bB >> ((OFF) + (H))) & 0xffu)) : 0u; \
        S2_STEP2(7, (OFF) + (H) + 7) S2_STEP2(6, (OFF) + (H) + 6)                                 \
        S2_STEP2(5, (OFF) + (H) + 5) S2_STEP2(4, (OFF) + (H) + 4)                                 \
        S2_STEP2(3, (OFF) + (H) + 3) S2_STEP2(2, (OFF) + (H) + 2)                                 \
        S2_STEP2(1, (OFF) + (H) + 1) S2_STEP2(0, (OFF) + (H) + 0)                                 \
        mA = (mA >> 16) & mkA;                                                                    \
        mB = (mB >> 16) & mkB;                                                                    \
        if (__builtin_expect((mA | mB) != 0, 0)) {                                                \
            if (mA)                                                                               \
                scan2_emit8<HK>(ev, abA, cntA, mA, hA, (H) ? WA.z : WA.x, (H) ? WA.w : WA.y,       \
                                bposA + (OFF) + (H), sA, ehi - sA, tk_base, eot_d, eot_k, dsh);   \
            if (mB)                                                                               \
                scan2_emit8<HK>(ev, abB, cntB, mB, hB, (H) ? WB.z : WB.x, (H) ? WB.w : WB.y,       \
                                bposB + (OFF) + (H), lo_r, sA - 1u - lo_r, tk_base, eot_d, eot_k, dsh); \
        }                                                                                         \
    }

#ifndef SCAN2_BLOCK
#define SCAN2_BLOCK 768
#endif
#ifndef SCAN2_WAVES
#define SCAN2_WAVES 6
#endif
template <bool HK, int NT = SCAN2_BLOCK>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == SCAN2_BLOCK ? SCAN2_WAVES : 4, NT == SCAN2_BLOCK ? SCAN2_WAVES : 4))) void k_scan2(
    const RulesDev R, const Geo g, const uint8_t* __restrict__ text, const uint32_t* __restrict__ words,
    const uint32_t* __restrict__ split, const uint32_t* __restrict__ lane_perm, Event* __restrict__ ev,
    uint32_t* __restrict__ lane_cnt, uint32_t* __restrict__ lane_st, const uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
    if (*err & ERR_ARGS) return;
    const int nd_words = R.SD * R.CDs / 2;
    const int nk_words = R.SK * R.CKs / 2;
    const uint32_t tk_base = SCAN_TD_BASE + (uint32_t)nd_words * 4;
    {
        const uint32_t* g_td = reinterpret_cast<const uint32_t*>(R.td);
        const uint32_t* g_tk = reinterpret_cast<const uint32_t*>(R.tk);
        uint32_t* d_td = smem32 + SCAN_TD_BASE / 4;
        uint32_t* d_tk = d_td + nd_words;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) smem32[i] = R.cmap4[i];
        for (int i = threadIdx.x; i < nd_words; i += blockDim.x) d_td[i] = g_td[i];
        for (int i = threadIdx.x; i < nk_words; i += blockDim.x) d_tk[i] = g_tk[i];
        uint32_t* d_sp = d_tk + nk_words;
        for (int i = threadIdx.x; i < 128; i += blockDim.x) d_sp[i] = scan_spread(2 * i) | scan_spread(2 * i + 1) << 16;
    }
    __syncthreads();
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;      // slot (lanes longest first)
    if (t >= g.n_chunks) return;
    const uint32_t c = lane_perm[t];
    const Lane L = g_lane(g, c);
    const uint32_t top = scan_top(g, L);
    const uint32_t end_r = (uint32_t)g_off(g, g.n_utt);
    uint32_t cnt = 0;
    if (top > L.lo) {
        uint32_t lo_r, len_r;
        emit_range(L, lo_r, len_r);
        const uint32_t ab = (uint32_t)ev_base(L, c);
        const uint32_t eot_d = SCAN_TD_BASE + 2u * (uint32_t)(R.CD - 1), eot_k = tk_base + 2u * (uint32_t)(R.CK - 1);
        const uint32_t spread = tk_base + (uint32_t)nk_words * 4;
        const uint32_t dsh = HK ? 0u : (uint32_t)R.dsh;
        const uint32_t sp = split[t];
        const uint32_t s = L.lo + (sp & 0xffffu);        // (lo when not split)
        const uint32_t abA = ab, abB = ab + (sp >> 16);
        // emission ranges: A [sA, ehi] ([s, e_hi] when split, the lane's own otherwise), B [lo_r, s - 1]
        const uint32_t sA = sp ? s : lo_r, ehi = lo_r + len_r;
        uint32_t ndA = 0, nkA = 0, pmA = 0xffffffffu, ndB = 0, nkB = 0, pmB = 0xffffffffu;
        if (L.chi) {             // (never split)
#if SCAN_INLINE_HALO
            const uint32_t hs = halo_state(R, g, text, L);
            lane_st[2 * c] = hs;
#else
            const uint32_t hs = lane_st[2 * c];
#endif
            ndA = hs & 0xffffu;
            nkA = hs >> 16;
            pmA = 0;
        }
        const uint32_t r0 = g.r0;
        const uintptr_t tpb = (uintptr_t)(text + g.base) - r0;
        const uint32_t hbA = (top - 1 + r0) >> 5, hb_lo = (L.lo + r0) >> 5;
        const uint32_t hs = sp ? (s + r0) >> 5 : hb_lo;
        const uint32_t nA = hbA - hs + 1, nB = sp ? hs - hb_lo + 1 : 0, hbB = hs;
        const uint32_t q_end = (end_r - 1 + r0) >> 4;             // last chunk with a batch byte
        const uint32_t n = g.n_chunks;           // (word rows * lanes < 2^32: rows < 2^8, lanes < 2^23)
        // the top half-block: its upper chunk only when it holds a batch byte (then every load is
        // unconditional: a finished chain re-reads its last half-block, its start bits forced to ones;
        // a chunk past the batch end is never read -- a top half-block's upper chunk is replaced by its
        // lower one, whose bytes then step only as garbage of a finished chain)
        // (uniform base + 32-bit offsets: the loads take the SGPR-base form, no 64-bit address VGPRs)
        const uint8_t* const tbase = reinterpret_cast<const uint8_t*>(tpb);
        auto ld = [&](uint32_t off) { return gload16_at(tbase, off); };
        auto hi16 = [&](uint32_t hb) { return hb * 32u + (2 * hb + 1 <= q_end ? 16u : 0u); };
        auto lo16 = [&](uint32_t hb) { return hb * 32u; };
        uint4 PA = make_uint4(0, 0, 0, 0);
        if (2 * hbA + 1 <= q_end) PA = ld(lo16(hbA) + 16);
        uint4 QA = ld(lo16(hbA)), PB = ld(hi16(hbB)), QB = ld(lo16(hbB));
        // (the lane's counts are re-derived per use: registers decide this kernel's occupancy)
#define LAST_A (nA - 1)
#define LAST_B (nB ? nB - 1 : 0u)
        uint32_t wA = words[t], wB = words[(uint32_t)HB_A * n + t];
        uint32_t nwA = words[min(1u, LAST_A) * n + t], nwB = words[(HB_A + min(1u, LAST_B)) * n + t];
        uint32_t cntA = 0, cntB = 0;
        for (uint32_t k = 0;; ++k) {
            const bool aliveA = k < nA, aliveB = k < nB;      // (lane masks: no VGPRs)
            const uint32_t bA = aliveA ? wA : 0xffffffffu, bB = aliveB ? wB : 0xffffffffu;
            const uint32_t ka = min(k + 1, LAST_A), kb = min(k + 1, LAST_B);
            const uint32_t bposA = 32u * (hbA - k) - r0, bposB = 32u * (hbB - k) - r0;
            S2_GROUP(PA, PB, 8, 16)
            S2_GROUP(PA, PB, 0, 16)
            PA = ld(hi16(hbA - ka));
            PB = ld(hi16(hbB - kb));
            S2_GROUP(QA, QB, 8, 0)
            S2_GROUP(QA, QB, 0, 0)
            QA = ld(lo16(hbA - ka));
            QB = ld(lo16(hbB - kb));
            wA = nwA;
            wB = nwB;
            nwA = words[min(k + 2, LAST_A) * n + t];
            nwB = words[(HB_A + min(k + 2, LAST_B)) * n + t];
            if (k + 1 >= max(nA, nB)) break;
        }
#undef LAST_A
#undef LAST_B
        // (the lane's id and cut flag re-read: nothing but the chains' state stays live across the loop)
        if (g.lanes[lane_perm[t]].z >> 31)                              // cut at lo: never split,
            lane_st[2 * lane_perm[t] + 1] = scan_state(ndA, nkA);       // A ended at byte lo
        if (cntB && abA + cntA < abB) {         // B's events behind A's (ascending: the target is lower)
            const uint2* src = reinterpret_cast<const uint2*>(ev + abB);
            uint2* dst = reinterpret_cast<uint2*>(ev + abA + cntA);
            for (uint32_t i = 0; i < cntB; i += 4) {
                uint2 x[4];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (i + r < cntB) x[r] = src[i + r];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (i + r < cntB) dst[i + r] = x[r];
            }
        }
        cnt = cntA + cntB;
    }
    lane_cnt[lane_perm[t]] = cnt;
}

// ---- k_scan_fix: stitching of cut rows.  A lane cut at hi scanned SCAN_HALO bytes past the cut from
// the start state; when that did not reproduce the state its right neighbour really ends with (a
// context longer than the halo: a long unbroken token), the lane is re-scanned from the true state.
// One workgroup per cut row: check every boundary, re-scan the mismatches (each from its right
// neighbour's state, which the same round may not change), then re-check only the boundaries left of
// a re-scanned lane until nothing changes.  Re-scans are rare and sequential per lane.
__device__ void rescan_lane(const RulesDev& R, const Geo& g, const uint8_t* __restrict__ text, uint32_t c,
                            uint32_t entry, Event* __restrict__ ev, uint32_t* __restrict__ lane_cnt,
                            uint32_t* __restrict__ lane_st) {
    const uint32_t* s_cmap = nullptr;        // LDS address 0 (k_scan layout)
    (void)s_cmap;
    const Lane L = g_lane(g, c);
    uint32_t lo_r, len_r;
    emit_range(L, lo_r, len_r);
    const uint32_t ab = (uint32_t)ev_base(L, c);
    const uint32_t nd_words = (uint32_t)(R.SD * R.CDs / 2);
    const uint32_t tk_base = SCAN_TD_BASE + nd_words * 4;
    const uint32_t eot_d = SCAN_TD_BASE + 2u * (uint32_t)(R.CD - 1), eot_k = tk_base + 2u * (uint32_t)(R.CK - 1);
    const uint8_t* tb = text + g.base;
    uint32_t nd = entry & 0xffffu, nk = entry >> 16, pm = 0;
    uint32_t cnt = 0;
    // utterance starts inside the lane, walked downwards
    const int64_t vmin = (int64_t)L.u0 + (L.clo ? 1 : 0);
    int64_t v = (int64_t)L.u1 - 1;
    while (v >= vmin && (g_off(g, (uint32_t)v) >= (int64_t)L.hi || g_off(g, (uint32_t)v + 1) == g_off(g, (uint32_t)v)))
        --v;
    for (int64_t b = (int64_t)L.hi - 1; b >= (int64_t)L.lo; --b) {
        const uint32_t cls = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>((size_t)(4u * tb[b]));
        const uint32_t x = cls;
        const uint32_t ad = ((nd & ~pm & 0xfffcu) << R.dsh) + (x & 0xffffu);
        const uint32_t ak = (nk & ~pm & 0xfffcu) + (R.SK > 1 ? (x >> 16) : tk_base);
        nd = lds_u16(ad);
        nk = lds_u16(ak);
        const bool st = v >= vmin && g_off(g, (uint32_t)v) == b;
        pm = st ? 0xffffffffu : 0u;
        if ((nd | nk) & 1u) scan_emit(ev, ab, cnt, (uint32_t)b + 1u, lo_r, len_r, ad, ak, tk_base);
        if (st) {
            if ((nd | nk) & 2u)
                scan_emit(ev, ab, cnt, (uint32_t)b, lo_r, len_r, ((nd & 0xfffcu) << R.dsh) + eot_d,
                          (nk & 0xfffcu) + eot_k, tk_base);
            --v;
            while (v >= vmin && g_off(g, (uint32_t)v + 1) == g_off(g, (uint32_t)v)) --v;     // empty rows
        }
    }
    lane_cnt[c] = cnt;
    lane_st[2 * c] = entry;
    if (L.clo) lane_st[2 * c + 1] = scan_state(nd, nk);
}

constexpr int FIX_Q = 512;
// LDS past the scan tables (the tables' entries are absolute LDS addresses, so the kernel declares no
// static LDS): queue, entry states, previous round's lanes, counters
constexpr size_t FIX_LDS = (3 * FIX_Q + 4) * 4;
#if !SCAN_INLINE_HALO && defined(SCAN_STREAMS) && SCAN_STREAMS > 1
// k_halo of group q runs on the engine stream after the fork; k_scan of that group on an aux stream
// that waits only on the fork: the scan would read halo states before k_halo writes them
#error "SCAN_STREAMS > 1 needs SCAN_INLINE_HALO (k_scan steps its own halo)"
#endif
#ifndef SCAN_STREAMS
#define SCAN_STREAMS 3                // streams for several SCAN groups' passes (config 5, wall per step, one box:
                                      // 1 / 2 / 3 -> 6.65 / 6.31 / 6.28 ms)
#endif

// All SCAN groups in one launch (blockIdx.y = group, its tables and arenas; one launch instead of one
// per group: config 5's seven idle launches cost 33 us per step).
__global__ __launch_bounds__(256) void k_scan_fix(const RulesDev* __restrict__ Rs, const uint32_t* __restrict__ lds_of,
                                                  const Geo g, const uint8_t* __restrict__ text,
                                                  const uint32_t* __restrict__ long_rows,
                                                  const uint32_t* __restrict__ long_count, Event* __restrict__ ev0,
                                                  uint64_t ev_stride, uint32_t* __restrict__ cnt0,
                                                  uint32_t* __restrict__ st0, uint64_t lane_stride,
                                                  uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
    if (blockIdx.x >= *long_count) return;
    const RulesDev R = Rs[blockIdx.y];
    const uint32_t scan_lds = lds_of[blockIdx.y];
    Event* __restrict__ ev = ev0 + blockIdx.y * ev_stride;
    uint32_t* __restrict__ lane_cnt = cnt0 + blockIdx.y * lane_stride;
    uint32_t* __restrict__ lane_st = st0 + 2 * blockIdx.y * lane_stride;
    uint32_t* s_q = smem32 + scan_lds / 4;
    uint32_t* s_e = s_q + FIX_Q;
    uint32_t* s_prev = s_e + FIX_Q;
    uint32_t& s_n = s_prev[FIX_Q];
    uint32_t& s_np = s_prev[FIX_Q + 1];
    uint32_t& s_full = s_prev[FIX_Q + 2];
    const uint32_t nrows = *long_count;
    if (blockIdx.x >= nrows || (*err & (ERR_ARGS | ERR_STITCH))) return;     // (STITCH: the row list overflowed)
    // the scan tables are staged in LDS only once a boundary needs a re-scan (the halo guesses are
    // almost always right: checking them needs no table, and a window step's ~1k short cut rows paid
    // a 62 KB table load per workgroup for nothing)
    bool staged = false;
    auto stage = [&]() {
        const int nd_words = R.SD * R.CDs / 2, nk_words = R.SK * R.CKs / 2;
        const uint32_t* g_td = reinterpret_cast<const uint32_t*>(R.td);
        const uint32_t* g_tk = reinterpret_cast<const uint32_t*>(R.tk);
        uint32_t* d_td = smem32 + SCAN_TD_BASE / 4;
        uint32_t* d_tk = d_td + nd_words;
        for (int i = threadIdx.x; i < 256; i += blockDim.x) smem32[i] = R.cmap4[i];
        for (int i = threadIdx.x; i < nd_words; i += blockDim.x) d_td[i] = g_td[i];
        for (int i = threadIdx.x; i < nk_words; i += blockDim.x) d_tk[i] = g_tk[i];
        __syncthreads();
        staged = true;
    };
    for (uint32_t ri = blockIdx.x; ri < nrows; ri += gridDim.x) {
        uint32_t ca, kb;
        int64_t s_r, e_r;
        row_lanes(g, long_rows[ri], ca, kb, s_r, e_r);
        // boundaries c | c + 1 for c in [ca, kb); round 1 checks all of them.  Every round fixes the
        // rightmost wrong boundary of each chain, so kb - ca + 1 rounds always suffice (the cap only
        // guards against a broken invariant: the batch then fails instead of spinning)
        bool all = true;
        for (uint32_t round = 0;; ++round) {
            if (round > kb - ca + 1) {
                if (threadIdx.x == 0) atomicOr(err, (uint32_t)ERR_STITCH);
                break;
            }
            if (threadIdx.x == 0) {
                s_n = 0;
                s_full = 0;
            }
            __syncthreads();
            if (all) {
                for (uint32_t c = ca + threadIdx.x; c < kb; c += blockDim.x) {
                    const uint32_t want = lane_st[2 * (c + 1) + 1];
                    if (lane_st[2 * c] != want) {
                        const uint32_t k = atomicAdd(&s_n, 1u);
                        if (k < FIX_Q) {
                            s_q[k] = c;
                            s_e[k] = want;
                        } else {
                            s_full = 1;
                        }
                    }
                }
            } else {
                for (uint32_t k = threadIdx.x; k < s_np; k += blockDim.x) {
                    const uint32_t c = s_prev[k];
                    if (c <= ca) continue;
                    const uint32_t b = c - 1;           // its left boundary: lane c's state changed
                    const uint32_t want = lane_st[2 * c + 1];
                    if (lane_st[2 * b] != want) {
                        const uint32_t q = atomicAdd(&s_n, 1u);
                        if (q < FIX_Q) {
                            s_q[q] = b;
                            s_e[q] = want;
                        } else {
                            s_full = 1;
                        }
                    }
                }
            }
            __syncthreads();
            const uint32_t n = min(s_n, (uint32_t)FIX_Q);
            if (n == 0 && !s_full) break;
            if (!staged) stage();                       // (n and s_full are block-uniform here)
            for (uint32_t k = threadIdx.x; k < n; k += blockDim.x)
                rescan_lane(R, g, text, s_q[k], s_e[k], ev, lane_cnt, lane_st);
            __syncthreads();
            for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) s_prev[k] = s_q[k];
            if (threadIdx.x == 0) s_np = n;
            all = s_full != 0;                          // an overflowed round re-checks everything
            __syncthreads();
        }
        __syncthreads();
    }
}
#undef SCAN_STEP8
#undef SCAN_GROUP8
#undef SCAN_CLASSES8
#undef SCAN_SUB

// ---------------------------------------------------------------------------- context (a11)
// segmented (by conversation run) scan of "latest agent row with a context hit"
struct SegV {
    uint32_t f;
    int32_t v;
};
__device__ __forceinline__ SegV seg_combine(SegV a, SegV b) {
    SegV r;
    r.f = a.f | b.f;
    r.v = b.f ? b.v : (a.v > b.v ? a.v : b.v);
    return r;
}

// Two passes over tiles of CTX_TILE rows, CTX_ITEMS consecutive rows per thread (all loads of a thread
// issued together): k_ctx_scan reduces each tile to its aggregate (and checks slots / ORDER);
// k_ctx_apply takes the tile's carry from the aggregates before it, re-scans the tile and applies the
// context per row.  No per-row scan values round-trip HBM.
constexpr int CTX_ITEMS = 8;
constexpr int CTX_THREADS = 256;
constexpr uint32_t CTX_TILE = CTX_ITEMS * CTX_THREADS;
static_assert(CTX_ITEMS == 8, "ctx_load's vector path reads 8 rows");

// the thread's rows [u0, u0 + CTX_ITEMS) clipped to n_utt: slot of row u0 - 1 .. u0 + CTX_ITEMS.
// VEC: slot / role are 16 / 8-byte aligned (host checked), so a full group is read with 16-byte loads
struct CtxRows {
    uint32_t sl[CTX_ITEMS + 2];      // sl[k + 1] = slot[u0 + k]; sl[0] = slot[u0 - 1]; past n_utt: ~0
    uint8_t role[CTX_ITEMS];
    int32_t kw[CTX_ITEMS];
};
template <bool VEC>
__device__ __forceinline__ void ctx_load(const uint32_t* __restrict__ slot, const uint8_t* __restrict__ role,
                                         const int32_t* __restrict__ kw, uint32_t n_utt, uint32_t u0, CtxRows& r) {
    r.sl[0] = u0 > 0 && u0 <= n_utt ? slot[u0 - 1] : 0xffffffffu;
    if (VEC && u0 + CTX_ITEMS <= n_utt) {
        const uint4 s0 = *reinterpret_cast<const uint4*>(slot + u0), s1 = *reinterpret_cast<const uint4*>(slot + u0 + 4);
        const uint2 ro = *reinterpret_cast<const uint2*>(role + u0);
        const int4 k0 = *reinterpret_cast<const int4*>(kw + u0), k1 = *reinterpret_cast<const int4*>(kw + u0 + 4);
        r.sl[1] = s0.x; r.sl[2] = s0.y; r.sl[3] = s0.z; r.sl[4] = s0.w;
        r.sl[5] = s1.x; r.sl[6] = s1.y; r.sl[7] = s1.z; r.sl[8] = s1.w;
        r.sl[9] = u0 + CTX_ITEMS < n_utt ? slot[u0 + CTX_ITEMS] : 0xfffffffeu;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r.role[k] = (uint8_t)(ro.x >> (8 * k));
            r.role[k + 4] = (uint8_t)(ro.y >> (8 * k));
        }
        r.kw[0] = k0.x; r.kw[1] = k0.y; r.kw[2] = k0.z; r.kw[3] = k0.w;
        r.kw[4] = k1.x; r.kw[5] = k1.y; r.kw[6] = k1.z; r.kw[7] = k1.w;
        return;
    }
#pragma unroll
    for (int k = 0; k <= CTX_ITEMS; ++k) r.sl[k + 1] = u0 + k < n_utt ? slot[u0 + k] : 0xfffffffeu;
#pragma unroll
    for (int k = 0; k < CTX_ITEMS; ++k) {
        const bool in = u0 + k < n_utt;
        r.role[k] = in ? role[u0 + k] : 0;
        r.kw[k] = in ? kw[u0 + k] : -1;
    }
}
__device__ __forceinline__ bool ctx_start(const CtxRows& r, uint32_t u0, int k) {
    return (u0 + k == 0) || r.sl[k] != r.sl[k + 1];
}
__device__ __forceinline__ SegV ctx_row(const CtxRows& r, uint32_t u0, int k) {
    SegV x;
    x.f = ctx_start(r, u0, k) ? 1u : 0u;
    x.v = (r.role[k] == PII_ROLE_AGENT && r.kw[k] >= 0) ? (int32_t)(u0 + k) : -1;
    return x;
}

// exclusive scan of one SegV per thread over the workgroup (prefix of thread 0 = identity)
__device__ __forceinline__ SegV ctx_block_excl(SegV x, SegV* wsum, SegV& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    SegV in = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        SegV o;
        o.f = __shfl_up(in.f, d);
        o.v = __shfl_up(in.v, d);
        if (lane >= d) in = seg_combine(o, in);
    }
    if (lane == 63) wsum[wid] = in;
    __syncthreads();
    SegV pre{0, -1};
    for (int w = 0; w < wid; ++w) pre = seg_combine(pre, wsum[w]);
    total = pre;
    for (int w = wid; w < CTX_THREADS / 64; ++w) total = seg_combine(total, wsum[w]);
    SegV ex;
    ex.f = __shfl_up(in.f, 1);
    ex.v = __shfl_up(in.v, 1);
    if (lane == 0) ex = SegV{0, -1};
    return seg_combine(pre, ex);
}

template <bool VEC>
__global__ __launch_bounds__(CTX_THREADS) void k_ctx_scan(const uint32_t* __restrict__ slot, const uint8_t* __restrict__ role,
                                                          const int32_t* __restrict__ kw, uint32_t n_utt, uint32_t n_slots,
                                                          int32_t* __restrict__ agg_v, uint32_t* __restrict__ agg_f,
                                                          uint32_t* __restrict__ stamp, uint32_t epoch,
                                                          uint32_t* __restrict__ err) {
    __shared__ SegV wsum[CTX_THREADS / 64];
    const uint32_t u0 = blockIdx.x * CTX_TILE + threadIdx.x * CTX_ITEMS;
    CtxRows r;
    ctx_load<VEC>(slot, role, kw, n_utt, u0, r);
    SegV x{0, -1};
    bool bad = false, order = false;
#pragma unroll
    for (int k = 0; k < CTX_ITEMS; ++k) {
        if (u0 + k >= n_utt) break;
        const uint32_t sl = r.sl[k + 1];
        bad |= sl >= n_slots;
        if (ctx_start(r, u0, k) && sl < n_slots) order |= atomicExch(&stamp[sl], epoch) == epoch;
        x = seg_combine(x, ctx_row(r, u0, k));
    }
    if (__any(bad)) {
        if ((threadIdx.x & 63) == 0) atomicOr(err, (uint32_t)ERR_SLOT);
    }
    if (__any(order)) {
        if ((threadIdx.x & 63) == 0) atomicOr(err, (uint32_t)ERR_ORDER);
    }
    SegV total;
    (void)ctx_block_excl(x, wsum, total);
    if (threadIdx.x == 0) {
        agg_v[blockIdx.x] = total.v;
        agg_f[blockIdx.x] = total.f;
    }
}

// latest hit of the run that continues into tile blk from the tiles before it (-1: none)
__device__ __forceinline__ int32_t ctx_carry(const int32_t* agg_v, const uint32_t* agg_f, int64_t blk) {
    for (int64_t b = blk - 1; b >= 0; --b) {
        if (agg_v[b] >= 0) return agg_v[b];
        if (agg_f[b]) return -1;
    }
    return -1;
}

// Per row: the context a CUSTOMER row uses (the latest AGENT hit before it in the same run, else the
// stored record, under the TTL), an AGENT row's own group; the last row of each run records the latest
// hit of the run (commit[u]) and appends u to the commit list (clist, *ncommit; read by k_ctx_commit).
template <bool VEC>
__global__ __launch_bounds__(CTX_THREADS) void k_ctx_apply(const uint32_t* __restrict__ slot, const uint8_t* __restrict__ role,
                                                           const int32_t* __restrict__ kw, const int64_t* __restrict__ ts,
                                                           uint32_t n_utt, uint32_t n_slots, int64_t ttl_us,
                                                           const int32_t* __restrict__ agg_v, const uint32_t* __restrict__ agg_f,
                                                           const int32_t* __restrict__ st_group, const int64_t* __restrict__ st_ts,
                                                           int16_t* __restrict__ ctx, int32_t* __restrict__ commit,
                                                           uint32_t* __restrict__ clist, uint32_t* __restrict__ ncommit,
                                                           int16_t* __restrict__ win_ctx) {
    __shared__ SegV wsum[CTX_THREADS / 64];
    __shared__ int32_t s_carry;
    __shared__ uint32_t s_n, s_base;
    if (threadIdx.x == 0) {
        s_carry = ctx_carry(agg_v, agg_f, blockIdx.x);
        s_n = 0;
    }
    const uint32_t u0 = blockIdx.x * CTX_TILE + threadIdx.x * CTX_ITEMS;
    CtxRows r;
    ctx_load<VEC>(slot, role, kw, n_utt, u0, r);
    SegV x{0, -1};
#pragma unroll
    for (int k = 0; k < CTX_ITEMS; ++k)
        if (u0 + k < n_utt) x = seg_combine(x, ctx_row(r, u0, k));
    SegV total;
    SegV run = ctx_block_excl(x, wsum, total);      // (the barrier inside also publishes s_carry)
    run = seg_combine(SegV{0, s_carry}, run);
    uint32_t lastm = 0;                                // bit k: row u0 + k ends a run (commit list)
    const bool full = VEC && u0 + CTX_ITEMS <= n_utt;
    int64_t tsv[CTX_ITEMS];
    if (full && ts) {
#pragma unroll
        for (int k = 0; k < CTX_ITEMS / 2; ++k) {
            const longlong2 t2 = *reinterpret_cast<const longlong2*>(ts + u0 + 2 * k);
            tsv[2 * k] = t2.x;
            tsv[2 * k + 1] = t2.y;
        }
    }
    int16_t cv[CTX_ITEMS], wv[CTX_ITEMS];
    // pass 1: each row's "latest hit strictly before it in the same run"; pass 2 issues every row's
    // record loads together (kw/ts of that hit, else the stored record), pass 3 decides
    int32_t prv[CTX_ITEMS];
    uint32_t need = 0;
#pragma unroll
    for (int k = 0; k < CTX_ITEMS; ++k) {
        prv[k] = ctx_start(r, u0, k) ? -1 : run.v;
        if (u0 + k < n_utt) run = seg_combine(run, ctx_row(r, u0, k));
        if (u0 + k < n_utt && (r.role[k] == PII_ROLE_CUSTOMER || win_ctx) && r.sl[k + 1] < n_slots) need |= 1u << k;
    }
    int32_t gg[CTX_ITEMS];
    int64_t tt[CTX_ITEMS];
#pragma unroll
    for (int k = 0; k < CTX_ITEMS; ++k) {
        gg[k] = -1;
        tt[k] = 0;
        if ((need >> k) & 1u) {
            if (prv[k] >= 0) {
                gg[k] = kw[prv[k]];
                tt[k] = ts ? ts[prv[k]] : 0;
            } else {
                gg[k] = st_group[r.sl[k + 1]];
                tt[k] = st_ts[r.sl[k + 1]];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < CTX_ITEMS; ++k) {
        const uint32_t u = u0 + k;
        if (u >= n_utt) break;
        const uint32_t sl = r.sl[k + 1];
        const int32_t prev = prv[k];
        const uint8_t ro = r.role[k];
        const int32_t kwu = r.kw[k];
        int16_t used = -1, live = -1;
        if ((need >> k) & 1u) {
            const int64_t now = ts ? (full ? tsv[k] : ts[u]) : 0;
            if (gg[k] >= 0 && (ts == nullptr || now - tt[k] < ttl_us)) live = (int16_t)gg[k];
            if (ro == PII_ROLE_CUSTOMER) used = live;
        }
        // the re-scan window of row u uses the context a request right after u would GET (main.py:403):
        // an AGENT row's own hit, else the live record
        wv[k] = (ro == PII_ROLE_AGENT && kwu >= 0) ? (int16_t)kwu : live;
        cv[k] = (ro == PII_ROLE_AGENT) ? (int16_t)kwu : used;
        if (!full) {
            if (win_ctx) win_ctx[u] = wv[k];
            ctx[u] = cv[k];
        }
        // last row of the run: the latest hit of the whole run (to be committed)
        const bool last = (u == n_utt - 1) || r.sl[k + 2] != sl;
        if (last && sl < n_slots) {
            commit[u] = (ro == PII_ROLE_AGENT && kwu >= 0) ? (int32_t)u : prev;
            lastm |= 1u << k;
        }
    }
    if (full) {
        auto pack = [](const int16_t (&a)[CTX_ITEMS]) {
            return make_uint4((uint16_t)a[0] | (uint32_t)(uint16_t)a[1] << 16, (uint16_t)a[2] | (uint32_t)(uint16_t)a[3] << 16,
                              (uint16_t)a[4] | (uint32_t)(uint16_t)a[5] << 16, (uint16_t)a[6] | (uint32_t)(uint16_t)a[7] << 16);
        };
        *reinterpret_cast<uint4*>(ctx + u0) = pack(cv);
        if (win_ctx) *reinterpret_cast<uint4*>(win_ctx + u0) = pack(wv);
    }
    const uint32_t nmine = (uint32_t)__builtin_popcount(lastm);
    uint32_t at = nmine ? atomicAdd(&s_n, nmine) : 0u;
    __syncthreads();
    if (threadIdx.x == 0 && s_n) s_base = atomicAdd(ncommit, s_n);
    __syncthreads();
    at += s_base;
    while (lastm) {
        clist[at++] = u0 + (uint32_t)__builtin_ctz(lastm);
        lastm &= lastm - 1u;
    }
}

// write the batch's context back (only when the whole call succeeded): one entry per conversation run
__global__ __launch_bounds__(256) void k_ctx_commit(const uint32_t* __restrict__ slot, const int32_t* __restrict__ kw,
                                                    const int64_t* __restrict__ ts, const uint32_t* __restrict__ clist,
                                                    const uint32_t* __restrict__ ncommit,
                                                    const int32_t* __restrict__ commit, const uint32_t* __restrict__ err,
                                                    int32_t* __restrict__ st_group, int64_t* __restrict__ st_ts) {
    if (*err != 0) return;
    const uint32_t n = *ncommit;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const uint32_t u = clist[k];
        const uint32_t sl = slot[u];
        const int32_t j = commit[u];
        if (j >= 0) {
            st_group[sl] = kw[j];
            st_ts[sl] = ts ? ts[j] : 0;
        }
    }
}

// ---------------------------------------------------------------------------------- resolve
// The sparse phase is data-parallel: divergent per-utterance loops serialise a wavefront, so the work
// is split into uniform phases over a queue of (candidate start, pattern) PAIRS.
//   k_pairs      per scan lane: decode its events; context keyword group of AGENT rows; append one
//                pair per (D event, pattern in the accept set) -- the lane's block is written back to
//                front so it ends up ascending by start, accept-set order within a start
//   k_pair_first per pair: anchored leftmost-first run -> end (or -1)      [lockstep DFA runs]
//   k_pair_eval  per matched pair: validator + hotword windows of the row's context variant -> likelihood
//   k_select     per scan lane: finditer skipping, exclusion, overlap resolution -> kept findings
struct EvLoc {         // where an event's candidates start (16 B: one dwordx4), one per event
    uint32_t u;        // utterance
    uint32_t s;        // candidate start, relative to the batch base
    uint32_t ustart;   // utterance start, relative to the batch base
    uint32_t uend;     // utterance end, relative to the batch base
};
struct PairRes {       // one (start, pattern) candidate (8 B); its FIRST end lives in pend[] (4 B)
    uint32_t ev;       // dense event index -> EvLoc
    uint16_t p;        // detector pattern
    int16_t lik;       // likelihood after validation + hotwords; -1 = invalid
};

// LDS images of rule tables, one per kernel (only what that kernel reads, so the pair kernels keep
// two 1024-thread workgroups per CU).  Sections are 16-byte aligned; off[] are byte offsets.
constexpr int IMG_MAX = 16;
struct LdsImage {
    uint32_t off[IMG_MAX];
    uint32_t total;    // bytes, multiple of 16
    uint32_t aux;      // index widths of the image's list tables (list_range): rule lists | exclusion lists << 3
};
// Per-(variant, type) hotword-rule and exclusion lists, deduplicated: key i -> list L = ix[i] (an index
// `w` bytes wide; w = 0: L = i, the undeduplicated global tables) -> ids[loff[L], loff[L + 1]).  Config 5
// has 23349 keys but 29 distinct rule lists and 2 exclusion lists: one byte per key instead of four,
// so the pair kernels' images keep their lists in LDS.
// (CL = false: the kernel instantiation for undeduplicated tables, the index not even tested -- the
// runtime test alone cost config 2's k_select 4 us)
template <bool CL>
__device__ __forceinline__ void list_range(const void* ix, uint32_t w, const uint32_t* loff, uint32_t i, uint32_t& r0,
                                           uint32_t& r1) {
    uint32_t L = i;
    if (CL) {
        if (w == 1) L = static_cast<const uint8_t*>(ix)[i];
        else if (w == 2) L = static_cast<const uint16_t*>(ix)[i];
        else if (w == 4) L = static_cast<const uint32_t*>(ix)[i];
    }
    r0 = loff[L];
    r1 = loff[L + 1];
}
enum { FI_TRANS, FI_CMAP, FI_DESC, FI_N };
enum { EV_TRANS, EV_CMAP, EV_HDESC, EV_HRULE, EV_DTYPE, EV_DVAL, EV_DLIK, EV_ROFF, EV_RIDS, EV_THOT, EV_RLOFF, EV_N };
// k_win_select: everything k_select reads + the HOT automata and the variants' hotword rule lists
enum { WS_TRANS, WS_CMAP, WS_HDESC, WS_HRULE, WS_DTYPE, WS_DLIK, WS_VEN, WS_VMIN, WS_DEX, WS_XOFF, WS_XIDS,
       WS_TOKOFF, WS_ROFF, WS_RIDS, WS_RLOFF, WS_XLOFF, WS_N };
enum { SE_DTYPE, SE_VEN, SE_VMIN, SE_DEX, SE_XOFF, SE_XIDS, SE_TOKOFF, SE_XLOFF, SE_N };

constexpr int PAIR_BLOCK = 1024;

constexpr int PAIR_WAVES = PAIR_BLOCK / 64;

// pair-queue segment of wavefront w of k_pair_first (and of its matched / continuation lists):
// [w*seg, (w+1)*seg), seg a multiple of 64
__device__ __forceinline__ uint64_t pair_segment(uint64_t n, uint32_t nwaves) {
    const uint64_t per = (n + nwaves - 1) / nwaves;
    return (per + 63) / 64 * 64;
}

struct FirstCont {     // a FIRST run still alive after its first window
    uint32_t i;        // pair
    uint32_t st;
    int32_t pos;       // next byte, relative to the utterance start
    int32_t last;
};
// what k_select reads of a matched pair, written by k_pair_eval next to the likelihood it computed
// (it lives in the continuation queue, free once k_pair_first is done; one 16-byte load instead of the pair record and then its event record)
struct SelRec {
    uint32_t u;        // utterance
    int32_t ps;        // start, relative to the utterance start
    uint32_t p;        // detector pattern | context variant << 16 (k_select needs no role / ctx load)
    int32_t lik;       // likelihood after validation + hotwords; -1 = invalid
};
static_assert(sizeof(SelRec) == sizeof(FirstCont), "SelRec aliases the FirstCont queue");

// Each wavefront first stages the offsets (u32, batch relative) and roles of the utterances its 64
// lanes cover into LDS with coalesced loads, so the per-lane walks (event -> utterance) read LDS
// instead of issuing dependent, uncoalesced global loads.  A wavefront whose lanes cover more than
// PAIRS_UCAP utterances (very short rows) walks global memory instead.
constexpr int PAIRS_BLOCK = 256;

// Two passes: k_pairs_flat<false> counts each lane's pairs (and records the AGENT rows' keyword
// groups), an exclusive scan of the counts gives every lane its block of the queue (lane order, no
// atomics), the write pass fills the blocks.
//
// MULTI (a rule set split over several SCAN groups, config 5): every group's k_scan pass wrote its
// own per-lane event list (descending position, arena g at ev + g * ev_stride), counted per group by
// the flat pass.  The write pass (k_pairs_merge) merges the lists by position, a tie going to the
// higher group first so that, the queue being filled back to front, group 0 (built-ins and
// excluders) comes first among one start's pairs, and writes the pairs.  (A per-lane walk
// of the merge -- one thread per lane, two dependent global loads per event -- took 1026 us at config
// 5; the rank form below 597 us.)
constexpr int SCAN_GROUPS_MAX = 8;
struct AccTabs {                 // per SCAN group, by D transition index:
    const uint16_t* accid[SCAN_GROUPS_MAX];   // global D accept-set id
    const uint16_t* npair[SCAN_GROUPS_MAX];   // pairs of that accept set
};

// MULTI write pass, rank form.  A wavefront owns MERGE_LPW consecutive lanes and stages every event
// of every group of its lanes in LDS (position, pairs | accept set, running pair count within the
// lane's group list), loaded flattened (64 events per load instruction, as in k_pairs_flat).  An
// event's place k in its lane's merged order (descending position, a tie going to the higher group
// -- the walk above) is its index in its own list plus, per other group, a binary search of that
// group's list in LDS; its first pair is the lane's top minus the pairs of every event up to and
// including it.  So no lane walks a serial chain of dependent global loads.  A wavefront whose
// lanes hold more than `evw_cap` events walks them one by one instead (merge_walk).  Shape (config 5,
// ~34 events per lane; lanes / staged events per wavefront -> us): 16/1024 1127, 8/512 696, 8/256 1698
// (most wavefronts walk), 4/384 690, 4/256 588, 2/256 769, 2/128 748.
#ifndef MERGE_LPW
#define MERGE_LPW 4
#endif
#ifndef MERGE_EVW
#define MERGE_EVW 256
#endif
constexpr int MERGE_WAVES = 4;
constexpr int MERGE_UCAP = 512;      // utterances of its lanes a wavefront stages
static_assert(MERGE_LPW <= 64 && (MERGE_LPW & (MERGE_LPW - 1)) == 0, "lanes per wavefront: a power of two <= 64");
static_assert(MERGE_EVW % 64 == 0, "staged events: whole 64-event chunks");

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// one lane's events in merged order, walked (the over-capacity fallback of k_pairs_merge)
__device__ void merge_walk(const Geo& g, const Event* __restrict__ ev, const uint32_t* __restrict__ lane_cnt,
                           uint32_t c, uint32_t n_groups, uint64_t ev_stride, uint32_t cnt_stride,
                           const AccTabs& acct, uint64_t top, uint64_t evb, EvLoc* __restrict__ evloc,
                           const uint32_t* __restrict__ acc_off, const uint16_t* __restrict__ acc_ids,
                           PairRes* __restrict__ pres) {
    const Lane L = g_lane(g, c);
    const uint64_t eb = ev_base(L, c);
    uint32_t gk[SCAN_GROUPS_MAX], gn[SCAN_GROUPS_MAX], hp[SCAN_GROUPS_MAX];
    uint32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < SCAN_GROUPS_MAX; ++q) {
        gk[q] = 0;
        gn[q] = (uint32_t)q < n_groups ? lane_cnt[(uint64_t)q * cnt_stride + c] : 0u;
        hp[q] = gn[q] ? ev[(uint64_t)q * ev_stride + eb].pos : 0u;
        cnt += gn[q];
    }
    uint64_t w = top;
    int64_t u = (int64_t)L.u1 - 1;
    int64_t s_u = g_off(g, (uint32_t)u), e_u = g_off(g, (uint32_t)u + 1);
    for (uint32_t k = 0; k < cnt; ++k) {
        uint32_t best = 0, bp = 0, kb = 0;
        bool any = false;
#pragma unroll
        for (int q = SCAN_GROUPS_MAX - 1; q >= 0; --q)
            if (gk[q] < gn[q] && (!any || hp[q] > bp)) {
                best = (uint32_t)q;
                bp = hp[q];
                any = true;
            }
        const uint16_t* accid = acct.accid[0];
        const uint16_t* npair = acct.npair[0];
#pragma unroll
        for (int q = 0; q < SCAN_GROUPS_MAX; ++q)
            if ((uint32_t)q == best) {
                kb = gk[q];
                accid = acct.accid[q];
                npair = acct.npair[q];
            }
        const uint64_t gb = (uint64_t)best * ev_stride + eb;
        const Event E = ev[gb + kb];
#pragma unroll
        for (int q = 0; q < SCAN_GROUPS_MAX; ++q)
            if ((uint32_t)q == best) {
                gk[q] = kb + 1;
                hp[q] = kb + 1 < gn[q] ? ev[gb + kb + 1].pos : 0u;
            }
        const int64_t pos = E.pos;
        while (pos < s_u) {
            --u;
            e_u = s_u;
            s_u = g_off(g, (uint32_t)u);
        }
        const uint32_t n = npair[E.sd];
        w -= n;
        if (n == 0) continue;
        const uint32_t a0 = acc_off[accid[E.sd]];
        for (uint32_t i = 0; i < n; ++i) {
            PairRes P;
            P.ev = (uint32_t)(evb + k);
            P.p = acc_ids[a0 + i];
            P.lik = -1;
            pres[w + i] = P;
        }
        EvLoc Lc;
        Lc.u = (uint32_t)u;
        Lc.s = (uint32_t)pos;
        Lc.ustart = (uint32_t)s_u;
        Lc.uend = (uint32_t)e_u;
        evloc[evb + k] = Lc;
    }
}

__global__ __launch_bounds__(MERGE_WAVES * 64) void k_pairs_merge(const Geo g, const Event* __restrict__ ev,
                                                           const uint32_t* __restrict__ lane_cnt,
                                                           EvLoc* __restrict__ evloc, PairRes* __restrict__ pres,
                                                           const uint32_t* __restrict__ acc_off,
                                                           const uint16_t* __restrict__ acc_ids,
                                                           uint64_t pair_cap, uint64_t ev_cap,
                                                           const uint64_t* __restrict__ lane_pair,
                                                           const uint64_t* __restrict__ lane_ev,
                                                           const uint32_t* __restrict__ lane_np,
                                                           uint32_t* __restrict__ err, uint32_t n_groups,
                                                           uint64_t ev_stride, uint32_t cnt_stride, const AccTabs acct,
                                                           uint32_t evw_cap) {
    __shared__ uint32_t s_pos[MERGE_WAVES][MERGE_EVW];
    __shared__ uint32_t s_na[MERGE_WAVES][MERGE_EVW];      // pairs | accept set << 16
    __shared__ uint32_t s_pn[MERGE_WAVES][MERGE_EVW];      // pairs of the lane's group list up to here
    __shared__ uint32_t s_lb[MERGE_WAVES][SCAN_GROUPS_MAX * MERGE_LPW + 1];   // list (q, l) start, q-major
    __shared__ uint32_t s_uo[MERGE_WAVES][MERGE_UCAP + 1];
    if (*err & ERR_ARGS) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t n_chunks = g.n_chunks;
    const uint32_t cw0 = (blockIdx.x * MERGE_WAVES + wv) * MERGE_LPW;
    if (cw0 >= n_chunks) return;                      // (no workgroup barriers below)
    const uint32_t nl = min((uint32_t)MERGE_LPW, n_chunks - cw0);
    const bool own = (uint32_t)lane < nl;             // lanes 0..nl-1 own scan lanes cw0 + lane
    const uint32_t c = cw0 + lane;
    const int64_t base = (int64_t)g.base;
    // the owners' lane records and per-group event counts, and the wavefront's row range: all loads
    // issued together (independent)
    uint32_t cq[SCAN_GROUPS_MAX], tot = 0, u0 = 0, u1 = 0;
    uint64_t eb = 0, top = 0, evb = 0;
    const uint32_t U0 = max(g.first_utt[cw0], 1u) - 1u, U1 = g.first_utt[cw0 + nl];
    Lane L{};
    uint64_t lp = 0, le = 0;
    uint32_t lnp = 0;
    if (own) {
        L = g_lane(g, c);
        lp = lane_pair[c];
        lnp = lane_np[c];
        le = lane_ev[c];
    }
#pragma unroll
    for (int r = 0; r < SCAN_GROUPS_MAX; ++r) {
        cq[r] = (own && (uint32_t)r < n_groups) ? lane_cnt[(uint64_t)r * cnt_stride + c] : 0u;
        tot += cq[r];
    }
    if (tot) {
        eb = ev_base(L, c);
        u0 = L.u0;
        u1 = L.u1;
        top = lp + lnp;
        evb = le;
    }
    const bool over = tot && (top > pair_cap || evb + tot > ev_cap);
    if (__any(over)) {
        if (lane == 0) atomicOr(err, (uint32_t)ERR_QUEUE);
        return;
    }
    // list starts, q-major over the wavefront's lanes (an exclusive scan of the counts)
    uint32_t* lbf = s_lb[wv];
    uint32_t T = 0;
#pragma unroll
    for (int r = 0; r < SCAN_GROUPS_MAX; ++r) {
        uint32_t incl = cq[r];
#pragma unroll
        for (int d = 1; d < MERGE_LPW; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
        if (lane < MERGE_LPW) lbf[r * MERGE_LPW + lane] = T + incl - cq[r];
        T += __shfl(incl, MERGE_LPW - 1);
    }
    if (T == 0) return;
    if (T > evw_cap) {                                // too many events to stage: walk them
        if (own && tot) merge_walk(g, ev, lane_cnt, c, n_groups, ev_stride, cnt_stride, acct, top, evb, evloc, acc_off,
                                     acc_ids, pres);
        return;
    }
    if (lane == 0) lbf[SCAN_GROUPS_MAX * MERGE_LPW] = T;
    // utterance offsets of the wavefront's lanes (rows [U0, U1], from one before the first lane's
    // first start: a cut row)
    const bool staged = U1 - U0 <= (uint32_t)MERGE_UCAP;
    uint32_t* so = s_uo[wv];
    if (staged)
        for (uint32_t k = lane; k <= U1 - U0; k += 64) so[k] = (uint32_t)((int64_t)g.offs[U0 + k] - base);
    auto uoff = [&](uint32_t u) { return staged ? so[u - U0] : (uint32_t)((int64_t)g.offs[u] - base); };
    uint32_t* sp = s_pos[wv];
    uint32_t* sa = s_na[wv];
    uint32_t* sn = s_pn[wv];
    wave_lds_sync();
    const uint32_t NL = n_groups * MERGE_LPW;
    // event f of the wavefront lies in list li = the last one whose start is <= f (an empty list
    // shares its start with the next one)
    auto list_of = [&](uint32_t f) {
        uint32_t li = 0;
#pragma unroll
        for (uint32_t st = SCAN_GROUPS_MAX * MERGE_LPW / 2; st >= 1; st >>= 1)
            if (li + st < NL && lbf[li + st] <= f) li += st;
        return li;
    };
    // stage every event (position, pairs | accept set), flattened over the lists; all 64-event
    // chunks of a wavefront in one round, their loads issued together
    constexpr int CH = MERGE_EVW / 64;
    for (uint32_t f0 = 0; f0 < T; f0 += CH * 64) {
        Event E[CH];
        uint32_t fq[CH];
#pragma unroll
        for (int r = 0; r < CH; ++r) {
            const uint32_t f = f0 + r * 64 + lane;
            const uint32_t li = list_of(f);
            const uint32_t q = li / MERGE_LPW, l = li % MERGE_LPW;
            const uint64_t o_eb = __shfl(eb, (int)l);
            fq[r] = q;
            E[r] = Event{};
            if (f < T) E[r] = ev[(uint64_t)q * ev_stride + o_eb + (f - lbf[li])];
        }
#pragma unroll
        for (int r = 0; r < CH; ++r) {
            const uint32_t f = f0 + r * 64 + lane;
            if (f < T) {
                const uint16_t* npair = acct.npair[0];
                const uint16_t* accid = acct.accid[0];
#pragma unroll
                for (int q = 1; q < SCAN_GROUPS_MAX; ++q)
                    if ((uint32_t)q == fq[r]) {
                        npair = acct.npair[q];
                        accid = acct.accid[q];
                    }
                sp[f] = E[r].pos;
                sa[f] = (uint32_t)npair[E[r].sd] | (uint32_t)accid[E[r].sd] << 16;
            }
        }
    }
    wave_lds_sync();
    // running pair count of every list (owners, in LDS)
    if (own && tot)
        for (uint32_t q = 0; q < n_groups; ++q) {
            const uint32_t b = lbf[q * MERGE_LPW + lane], n = lbf[q * MERGE_LPW + lane + 1] - b;
            uint32_t run = 0;
            for (uint32_t i = 0; i < n; ++i) {
                run += sa[b + i] & 0xffffu;
                sn[b + i] = run;
            }
        }
    wave_lds_sync();
    // every event's merged rank and first pair, flattened over the lists; then the chunk's (start,
    // pattern) pairs, wave-cooperative as in k_pairs_flat (a separate expansion kernel reading an
    // 8-byte record per event: merge 599 + expand 115 us against 689 us fused).
    // (Permuting the event records through LDS so that their stores land in slot order measured
    // slower: 597 -> 617 us at config 5.)
    for (uint32_t f0 = 0; f0 < T; f0 += 64) {
        const uint32_t f = f0 + lane;
        const bool act = f < T;
        const uint32_t li = list_of(f);
        const uint32_t q = li / MERGE_LPW, ow = li % MERGE_LPW;
        const uint64_t o_top = __shfl(top, (int)ow), o_evb = __shfl(evb, (int)ow);
        const uint32_t o_u0 = __shfl(u0, (int)ow), o_u1 = __shfl(u1, (int)ow);
        uint32_t n = 0, first = 0, a0 = 0, evi = 0;
        if (act) {
            const uint32_t pos = sp[f], na = sa[f];
            uint32_t k = f - lbf[li];                      // index in its own list
            uint32_t pn = sn[f];                           // pairs up to and including it, own list
            for (uint32_t q2 = 0; q2 < n_groups; ++q2) {   // events of q2 placed before this one
                if (q2 == q) continue;
                const uint32_t b2 = lbf[q2 * MERGE_LPW + ow];
                uint32_t lo = 0, hi = lbf[q2 * MERGE_LPW + ow + 1] - b2;
                while (lo < hi) {
                    const uint32_t m = (lo + hi) >> 1;
                    const uint32_t p2 = sp[b2 + m];
                    if (p2 > pos || (p2 == pos && q2 > q)) lo = m + 1;
                    else hi = m;
                }
                k += lo;
                if (lo) pn += sn[b2 + lo - 1];
            }
            n = na & 0xffffu;
            first = (uint32_t)(o_top - pn);
            evi = (uint32_t)(o_evb + k);
            if (n) {
                a0 = acc_off[na >> 16];
                uint32_t lo = o_u0, hi = o_u1 - 1;       // the event's row: last u with start <= pos
                while (lo < hi) {
                    const uint32_t m = (lo + hi + 1) >> 1;
                    if (uoff(m) <= pos) lo = m;
                    else hi = m - 1;
                }
                EvLoc Lc;
                Lc.u = lo;
                Lc.s = pos;
                Lc.ustart = uoff(lo);
                Lc.uend = uoff(lo + 1);
                evloc[evi] = Lc;
            }
        }
        uint32_t ein = n;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(ein, d);
            if (lane >= d) ein += o;
        }
        const uint32_t etot = __shfl(ein, 63);
        for (uint32_t p0 = 0; p0 < etot; p0 += 64) {
            const uint32_t pq = p0 + lane;
            int lo = 0;                                   // the pair's event: first lane with ein > pq
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1)
                if (__shfl(ein, lo + st - 1) <= pq) lo += st;
            const uint32_t p_incl = __shfl(ein, lo), p_n = __shfl(n, lo);
            const uint32_t p_first = __shfl(first, lo), p_a0 = __shfl(a0, lo), p_ev = __shfl(evi, lo);
            if (pq < etot) {
                const uint32_t i = pq - (p_incl - p_n);
                PairRes P;
                P.ev = p_ev;
                P.p = acc_ids[p_a0 + i];
                P.lik = -1;
                pres[p_first + i] = P;
            }
        }
    }
}

// One SCAN group: the same two passes, wave-cooperative.  A wavefront's 64 lanes own consecutive
// blocks of the event numbering (lane_ev), so their events are processed as one flattened list, 64
// at a time: event f belongs to the first lane whose inclusive event count exceeds f (a 6-step
// shuffle search), its utterance is found by a binary search over that lane's staged utterance
// offsets, and every per-event record is written at E0 + f -- 64 neighbouring records per store
// instead of record k of 64 lanes (the per-lane walk is a serial chain of dependent loads, and its
// stores land in 64 different lines).  Pair numbering per lane is back to front (ascending by start,
// as the per-lane form): a segmented scan of the events' pair counts plus each lane's running total.
// Keyword groups of AGENT rows are merged with atomic min (init: k_chunk_index).
template <bool WRITE>
__global__ __launch_bounds__(PAIRS_BLOCK) void k_pairs_flat(const RulesDev R, const Geo g,
                                                    const Event* __restrict__ ev, const uint32_t* __restrict__ lane_cnt,
                                                    const uint8_t* __restrict__ role, int32_t* __restrict__ kw,
                                                    EvLoc* __restrict__ evloc,
                                                    uint64_t pair_cap, uint64_t ev_cap,
                                                    const uint64_t* __restrict__ lane_pair,
                                                    const uint64_t* __restrict__ lane_ev,
                                                    uint32_t* __restrict__ lane_np, uint32_t* __restrict__ err,
                                                    PairRes* __restrict__ pres, const AccTabs acct,
                                                    uint32_t n_groups, uint64_t ev_stride, uint32_t cnt_stride,
                                                    uint32_t* __restrict__ lane_evn) {
    __shared__ uint32_t s_off[PAIRS_BLOCK / 64][PAIRS_UCAP + 1];
    __shared__ uint8_t s_role[PAIRS_BLOCK / 64][PAIRS_UCAP];
    __shared__ uint32_t s_aoff[257];
    __shared__ uint16_t s_aids[2048];
    if (*err & ERR_ARGS) return;
    // WRITE: the accept sets' pattern lists (the pair expansion below), staged when small
    const uint32_t n_dacc = R.n_dacc;
    const bool small = WRITE && n_dacc < 256 && R.d_acc_off[n_dacc] <= 2048;
    if (small) {
        for (uint32_t i = threadIdx.x; i <= n_dacc; i += blockDim.x) s_aoff[i] = R.d_acc_off[i];
        for (uint32_t i = threadIdx.x; i < R.d_acc_off[n_dacc]; i += blockDim.x) s_aids[i] = R.d_acc_ids[i];
    }
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t n_chunks = g.n_chunks;
    const uint64_t* __restrict__ offs = g.offs;
    const int64_t base = (int64_t)g.base;
    const uint32_t cw0 = c - lane;
    const uint32_t cw1 = min(cw0 + 64, n_chunks);
    const uint32_t U0 = cw0 < n_chunks ? max(g.first_utt[cw0], 1u) - 1u : 0u;
    const uint32_t U1 = cw0 < n_chunks ? g.first_utt[cw1] : 0u;
    const bool staged = U1 - U0 <= (uint32_t)PAIRS_UCAP;
    uint32_t* so = s_off[wv];
    uint8_t* sr = s_role[wv];
    if (staged && cw0 < n_chunks) {
        for (uint32_t k = lane; k <= U1 - U0; k += 64) so[k] = (uint32_t)((int64_t)offs[U0 + k] - base);
        if (!WRITE)
            for (uint32_t k = lane; k < U1 - U0; k += 64) sr[k] = role[U0 + k];
    }
    __syncthreads();
    if (cw0 >= n_chunks) return;
    auto uoff = [&](uint32_t u) { return staged ? so[u - U0] : (uint32_t)((int64_t)offs[u] - base); };
    const bool valid = c < n_chunks;
    // count pass over several SCAN groups (config 5): blockIdx.y = group, its own event arena and
    // per-transition pair counts; only group 0 carries the keyword automaton.  The lanes' pair counts
    // add up over the groups (lane_np is zeroed first), group 0 writes the lanes' total event counts.
    const uint32_t q = WRITE ? 0u : blockIdx.y;
    const uint16_t* __restrict__ npair = q ? acct.npair[q] : R.d_npair;
    if (!WRITE && n_groups > 1 && q == 0 && valid) {
        uint32_t tot = 0;
        for (uint32_t k = 0; k < n_groups; ++k) tot += lane_cnt[(uint64_t)k * cnt_stride + c];
        lane_evn[c] = tot;
    }
    ev += (uint64_t)q * ev_stride;
    lane_cnt += (uint64_t)q * cnt_stride;
    const uint32_t cnt = valid ? lane_cnt[c] : 0u;
    uint32_t eb = 0, u0 = 0, u1 = 0;                      // the lane's arena, utterances [u0, u1)
    if (cnt) {
        const Lane L = g_lane(g, c);
        eb = (uint32_t)ev_base(L, c);
        u0 = L.u0;
        u1 = L.u1;
    }
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    const uint32_t total = __shfl(incl, 63), excl = incl - cnt;
    uint64_t E0 = 0, top = 0;            // WRITE: the wave's first event record; lane: its last pair + 1
    if (WRITE) {
        E0 = lane_ev[cw0];
        top = valid ? lane_pair[c] + lane_np[c] : 0;
        const bool over = (valid && top > pair_cap) || E0 + total > ev_cap;
        if (__any(over)) {
            if (lane == 0) atomicOr(err, (uint32_t)ERR_QUEUE);
            return;
        }
    }
    uint32_t run = 0;                                     // lane: pairs of its events handled so far
    // event f's owner (first lane with incl > f) and record; the next chunk's are loaded while this
    // chunk is processed (one dependent load less per chunk)
    auto owner_of = [&](uint32_t f) {
        int ow = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
            const uint32_t v = __shfl(incl, ow + step - 1);
            if (v <= f) ow += step;
        }
        return ow;
    };
    auto event_of = [&](uint32_t f, int ow) {
        const uint32_t o_ex = __shfl(excl, ow), o_eb = __shfl(eb, ow);
        Event E{};
        if (f < total) E = ev[(uint64_t)o_eb + (f - o_ex)];
        return E;
    };
    int ow_n = owner_of(lane);
    Event E_n = event_of(lane, ow_n);
    for (uint32_t f0 = 0; f0 < total; f0 += 64) {
        const uint32_t f = f0 + lane;
        const bool act = f < total;
        const int ow = ow_n;
        const Event E = E_n;
        if (f0 + 64 < total) {
            ow_n = owner_of(f + 64);
            E_n = event_of(f + 64, ow_n);
        }
        const uint32_t o_ex = __shfl(excl, ow);
        const uint32_t o_u0 = __shfl(u0, ow), o_u1 = __shfl(u1, ow), o_run = __shfl(run, ow);
        const uint64_t o_top = WRITE ? __shfl(top, ow) : 0;
        (void)o_ex;
        uint32_t n = 0, acc = 0, u = 0, kg = (uint32_t)KW_NONE;
        if (act) {
            n = npair[E.sd];
            if (WRITE) acc = R.d_accid[E.sd];
            else if (q == 0) kg = R.k_grp[E.sk];
            // the event's row (last u with start <= pos): the count pass needs it only for a keyword
            if (WRITE || kg != (uint32_t)KW_NONE) {
                uint32_t lo = o_u0, hi = o_u1 - 1;
                while (lo < hi) {
                    const uint32_t m = (lo + hi + 1) >> 1;
                    if (uoff(m) <= E.pos) lo = m;
                    else hi = m - 1;
                }
                u = lo;
            }
        }
        // pairs of the owner's events up to and including this one (segmented inclusive scan)
        uint32_t sc = n;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(sc, d);
            const int oo = __shfl_up(ow, d);
            if (lane >= d && oo == ow) sc += o;
        }
        if (act) {
            if (WRITE) {
                if (n) {
                    EvLoc Lc;
                    Lc.u = u;
                    Lc.s = E.pos;
                    Lc.ustart = uoff(u);
                    Lc.uend = uoff(u + 1);
                    evloc[E0 + f] = Lc;
                }
            } else if (q == 0) {
                if (kg != (uint32_t)KW_NONE && (staged ? sr[u - U0] : role[u]) == PII_ROLE_AGENT)
                    atomicMin(reinterpret_cast<unsigned int*>(kw + u), kg);
            }
        }
        if (WRITE) {
            // the chunk's (start, pattern) pairs, wave-cooperative: numbered 0..tot-1 by a scan of the
            // events' counts, lane q writes pair q, q + 64, ... (its event found by a 6-step search), so
            // one store instruction writes neighbouring records (the pair blocks of one lane's events
            // are adjacent)
            const uint32_t en = act ? n : 0u;
            const uint32_t efirst = act ? (uint32_t)(o_top - (o_run + sc)) : 0u;
            const uint32_t ea0 = en ? (small ? s_aoff[acc] : R.d_acc_off[acc]) : 0u;
            uint32_t ein = en;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(ein, d);
                if (lane >= d) ein += o;
            }
            const uint32_t etot = __shfl(ein, 63);
            for (uint32_t q0 = 0; q0 < etot; q0 += 64) {
                const uint32_t q = q0 + lane;
                int lo = 0;
#pragma unroll
                for (int step = 32; step >= 1; step >>= 1) {
                    const uint32_t v = __shfl(ein, lo + step - 1);
                    if (v <= q) lo += step;
                }
                const uint32_t p_incl = __shfl(ein, lo), p_n = __shfl(en, lo);
                const uint32_t p_a0 = __shfl(ea0, lo), p_first = __shfl(efirst, lo);
                if (q < etot) {
                    const uint32_t i = q - (p_incl - p_n);
                    PairRes P;
                    P.ev = (uint32_t)(E0 + f0 + lo);
                    P.p = small ? s_aids[p_a0 + i] : R.d_acc_ids[p_a0 + i];
                    P.lik = -1;
                    pres[p_first + i] = P;
                }
            }
        }
        // each lane adds its events' pairs of this chunk (the scan value at its last slot here)
        const bool here = cnt && incl > f0 && excl < f0 + 64;
        const int last = here ? (int)(min(incl, f0 + 64) - 1 - f0) : 0;
        const uint32_t add = __shfl(sc, last);
        if (here) run += add;
    }
    if (!WRITE && valid) {
        if (n_groups > 1) atomicAdd(lane_np + c, run);
        else lane_np[c] = run;
    }
}

// GI: the image is too large for LDS (config-5 rule sets: every FIRST automaton of 500+ types) and
// is read in place from global memory (L2-resident), the kernel launched without dynamic LDS
template <bool GI = false>
__device__ __forceinline__ const uint8_t* load_image(const uint4* __restrict__ img, uint32_t total, uint4* lds4) {
    if (GI) return reinterpret_cast<const uint8_t*>(img);
    for (uint32_t i = threadIdx.x; i < total / 16; i += blockDim.x) lds4[i] = img[i];
    __syncthreads();
    return reinterpret_cast<const uint8_t*>(lds4);
}

// per pair: anchored leftmost-first run.  Each wavefront owns one contiguous segment of the queue
// (no workgroup barriers while it runs) and compacts, by ballot, its matched pairs into the same
// segment of `matched` and the runs still alive after one 16-byte window into the same segment of
// `cont`.  The workgroup then finishes all its continuations densely, so one long run no longer holds
// 63 idle lanes; their matches are appended through LDS counters.
//
// GI (the image past LDS, read in place from L2): the automata of the first `p_hot` patterns (the
// shipped built-in types come first: half of config 5's pairs) are copied into LDS as a second image
// `himg`, and a pair of those patterns steps them there -- fewer L2 requests, the bound of this
// kernel at config 5.  (Pointers are then generic: a lane's loads go to LDS or L2 by its pattern.)
template <bool GI>
__global__ __launch_bounds__(PAIR_BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pair_first(const uint4* __restrict__ img, const LdsImage li,
                                                           const uint8_t* __restrict__ text0,
                                                           const uint64_t* __restrict__ offs,
                                                           const unsigned long long* __restrict__ pair_count,
                                                           uint64_t pair_cap, const EvLoc* __restrict__ evloc,
                                                           const PairRes* __restrict__ pres,
                                                           int32_t* __restrict__ pend, uint32_t* __restrict__ matched,
                                                           FirstCont* __restrict__ cont,
                                                           uint32_t* __restrict__ mcount,
                                                           const uint32_t* __restrict__ err,
                                                           const uint4* __restrict__ himg, const LdsImage hli,
                                                           uint32_t p_hot) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    __shared__ uint32_t s_mc[PAIR_WAVES], s_cc[PAIR_WAVES + 1];
    if (*err & ERR_ABORT) {
        if (threadIdx.x < PAIR_WAVES) mcount[blockIdx.x * PAIR_WAVES + threadIdx.x] = 0;
        return;
    }
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    const Pool pool{reinterpret_cast<const uint16_t*>(lb + li.off[FI_TRANS]), lb + li.off[FI_CMAP]};
    const int32_t* fdesc = reinterpret_cast<const int32_t*>(lb + li.off[FI_DESC]);
    Pool hpool = pool;
    const int32_t* hdesc = fdesc;
    if (GI && p_hot) {
        const uint8_t* hb = load_image<false>(himg, hli.total, lds4);
        hpool = Pool{reinterpret_cast<const uint16_t*>(hb + hli.off[FI_TRANS]), hb + hli.off[FI_CMAP]};
        hdesc = reinterpret_cast<const int32_t*>(hb + hli.off[FI_DESC]);
    }
    // a pattern's automaton: the LDS copy for the leading patterns (GI), else the image's
    auto tabs = [&](uint32_t p, Pool& pl, const int32_t*& d) {
        const bool h = GI && p < p_hot && hdesc[8 * p + 3] != 0;
        pl = h ? hpool : pool;
        d = (h ? hdesc : fdesc) + 8 * p;
    };
    const uint64_t n = min((uint64_t)*pair_count, pair_cap);
    const uint8_t* text = text0 + offs[0];     // pair positions are relative to the batch base
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * PAIR_WAVES + wave;
    const uint64_t seg = pair_segment(n, gridDim.x * PAIR_WAVES);
    const uint64_t lo = gw * seg, hi = min(n, lo + seg);
    const uint64_t lanemask = (1ull << lane) - 1;
    uint32_t mc = 0, cc = 0;
    for (uint64_t b = lo; b < hi; b += 64) {
        const uint64_t i = b + lane;
        int e = -1;
        FirstState r;
        if (i < hi) {
            const PairRes P = pres[i];
            const EvLoc L = evloc[P.ev];
            Pool pl;
            const int32_t* d;
            tabs(P.p, pl, d);
            e = first_begin(pl, d, text + L.ustart, (int)(L.s - L.ustart), (int)(L.uend - L.ustart), r);
            pend[i] = e < 0 ? -1 : e;                 // still-running runs (-2) are completed below
        }
        const uint64_t mm = __ballot(e >= 0), mcn = __ballot(e == -2);
        if (e >= 0) matched[lo + mc + __popcll(mm & lanemask)] = (uint32_t)i;
        if (e == -2) {
            FirstCont C;
            C.i = (uint32_t)i;
            C.st = r.st;
            C.pos = r.pos;
            C.last = r.last;
            cont[lo + cc + __popcll(mcn & lanemask)] = C;
        }
        mc += __popcll(mm);
        cc += __popcll(mcn);
    }
    if (lane == 0) {
        s_mc[wave] = mc;
        s_cc[wave] = cc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < PAIR_WAVES; ++w) {
            const uint32_t c = s_cc[w];
            s_cc[w] = run;
            run += c;
        }
        s_cc[PAIR_WAVES] = run;
    }
    __syncthreads();
    // continuations of the whole workgroup, densely
    const uint32_t total = s_cc[PAIR_WAVES];
    for (uint32_t k = threadIdx.x; k < total; k += PAIR_BLOCK) {
        int w = 0;
        while (w + 1 < PAIR_WAVES && s_cc[w + 1] <= k) ++w;
        const uint64_t wlo = (uint64_t)(blockIdx.x * PAIR_WAVES + w) * seg;
        const FirstCont C = cont[wlo + (k - s_cc[w])];
        const PairRes P = pres[C.i];
        const EvLoc L = evloc[P.ev];
        FirstState r{C.st, C.pos, C.last};
        Pool pl;
        const int32_t* d;
        tabs(P.p, pl, d);
        const int e = first_finish(pl, d, text + L.ustart, (int)(L.uend - L.ustart), r);
        if (e >= 0) {
            pend[C.i] = e;
            matched[wlo + atomicAdd(&s_mc[w], 1u)] = C.i;
        }
    }
    __syncthreads();
    if (threadIdx.x < PAIR_WAVES) mcount[blockIdx.x * PAIR_WAVES + threadIdx.x] = s_mc[threadIdx.x];
}

// the eval image's tables (k_pair_eval)
struct EvalTabs {
    Pool pool;
    const int32_t* hdesc;
    const int32_t* hrule;
    const uint16_t* dtype;
    const uint8_t* dval;
    const uint8_t* dlik;
    const void* rix;          // rule lists (list_range)
    uint32_t rw;
    const uint32_t* rloff;
    const uint16_t* rids;
};
__device__ __forceinline__ EvalTabs eval_tabs(const uint8_t* lb, const LdsImage& li) {
    EvalTabs E;
    E.pool = Pool{reinterpret_cast<const uint16_t*>(lb + li.off[EV_TRANS]), lb + li.off[EV_CMAP]};
    E.hdesc = reinterpret_cast<const int32_t*>(lb + li.off[EV_HDESC]);
    E.hrule = reinterpret_cast<const int32_t*>(lb + li.off[EV_HRULE]);
    E.dtype = reinterpret_cast<const uint16_t*>(lb + li.off[EV_DTYPE]);
    E.dval = lb + li.off[EV_DVAL];
    E.dlik = lb + li.off[EV_DLIK];
    E.rix = lb + li.off[EV_ROFF];
    E.rw = li.aux & 7u;
    E.rloff = reinterpret_cast<const uint32_t*>(lb + li.off[EV_RLOFF]);
    E.rids = reinterpret_cast<const uint16_t*>(lb + li.off[EV_RIDS]);
    return E;
}

// likelihood of the match [s, e) of pattern p in row t0[0, L) under context variant v: the validator,
// then every hotword rule of (v, type) in order (window_before / window_after, fixed / relative); -1
// when the validator rejects it
template <bool CL>
__device__ __forceinline__ int pair_lik(const EvalTabs& E, int T, const uint8_t* t0, int L, int s, int e, int p,
                                        int v) {
    if (!validate(E.dval[p], t0 + s, e - s)) return -1;
    const int t = E.dtype[p];
    int lik = E.dlik[p];
    uint32_t r0, r1;
    list_range<CL>(E.rix, E.rw, E.rloff, (uint32_t)(v * T + t), r0, r1);
    for (uint32_t q = r0; q < r1; ++q) {
        const int h = E.rids[q];
        const int wb = E.hrule[4 * h], wa = E.hrule[4 * h + 1];
        const int fixed = E.hrule[4 * h + 2], rel = E.hrule[4 * h + 3];
        bool hit = false;
        // window_before, then window_after: one call site (one copy of the runner's registers)
#pragma unroll 1
        for (int side = 0; side < 2 && !hit; ++side) {
            const int w = side ? wa : wb;
            if (w > 0) {
                const int lo = side ? e : (s - w > 0 ? s - w : 0);
                const int hi = side ? (e + w < L ? e + w : L) : s;
                hit = hot_run(E.pool, E.hdesc + 8 * h, t0, lo, hi);
            }
        }
        if (hit) {
            if (fixed) {
                lik = fixed;
            } else {
                lik += rel;
                lik = lik < 1 ? 1 : (lik > 5 ? 5 : lik);
            }
        }
    }
    return lik;
}

// per matched pair: validator + hotword windows of the row's context variant -> likelihood
// RG: the image omits the per-(variant, type) rule lists (config 5's are 107 KB: with them the image
// leaves room for one 1024-thread workgroup per CU); they are read from global memory (L2) instead
template <bool GI, bool RG = false, bool CL = false>
__global__ __launch_bounds__(PAIR_BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pair_eval(const uint4* __restrict__ img, const LdsImage li, int T,
                                                          const uint8_t* __restrict__ text0,
                                                          const uint64_t* __restrict__ offs,
                                                          const uint8_t* __restrict__ role,
                                                          const int16_t* __restrict__ ctx,
                                                          const unsigned long long* __restrict__ pair_count,
                                                          uint64_t pair_cap, const uint32_t* __restrict__ matched,
                                                          const uint32_t* __restrict__ mcount, uint32_t nseg,
                                                          const EvLoc* __restrict__ evloc,
                                                          const int32_t* __restrict__ pend,
                                                          const PairRes* __restrict__ pres, SelRec* __restrict__ sel,
                                                          const uint32_t* __restrict__ g_roff,
                                                          const uint16_t* __restrict__ g_rids, uint32_t split) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    EvalTabs E = eval_tabs(lb, li);
    if (RG) {
        E.rix = nullptr;
        E.rw = 0;
        E.rloff = g_roff;
        E.rids = g_rids;
    }
    const uint8_t* text = text0 + offs[0];
    __shared__ uint32_t s_mp[PAIR_WAVES + 1];
    const uint64_t seg = pair_segment(min((uint64_t)*pair_count, pair_cap), nseg * PAIR_WAVES);
    // work unit gj = part (gj % split) of k_pair_first workgroup gj / split's matched pairs: with split
    // > 1 the grid runs several rounds of workgroups, so one whose pairs took long no longer leaves its
    // CU half empty until the kernel ends (one round: 4.6 of 8 waves/SIMD on average)
    for (uint32_t gj = blockIdx.x; gj < nseg * split; gj += gridDim.x) {
        const uint32_t g = gj / split, part = gj % split;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int w = 0; w < PAIR_WAVES; ++w) {
                s_mp[w] = run;
                run += mcount[g * PAIR_WAVES + w];
            }
            s_mp[PAIR_WAVES] = run;
        }
        __syncthreads();
        const uint32_t m = s_mp[PAIR_WAVES];
        const uint32_t k0 = (uint32_t)((uint64_t)m * part / split), k1 = (uint32_t)((uint64_t)m * (part + 1) / split);
        for (uint32_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) {
            int w = 0;
            while (w + 1 < PAIR_WAVES && s_mp[w + 1] <= k) ++w;
            const uint32_t i = matched[(uint64_t)(g * PAIR_WAVES + w) * seg + (k - s_mp[w])];
            const PairRes P = pres[i];
            const EvLoc Lc = evloc[P.ev];
            const uint8_t* t0 = text + Lc.ustart;
            const int L = (int)(Lc.uend - Lc.ustart);
            const int s = (int)(Lc.s - Lc.ustart), e = pend[i];
            const uint32_t u = Lc.u;
            const int v = (role[u] == PII_ROLE_CUSTOMER && ctx[u] >= 0) ? ctx[u] + 1 : 0;
            const int lik = pair_lik<CL>(E, T, t0, L, s, e, P.p, v);
            SelRec r;
            r.u = Lc.u;
            r.ps = s;
            r.p = P.p | (uint32_t)v << 16;          // k_select takes the row's variant from here
            r.lik = lik;
            sel[i] = r;
        }
    }
}

constexpr int LIVE = 5;            // register-resident "previous match end" slots per lane

// bit j: entry g0 + j of an aligned 16-entry pend[] group is a match (>= 0) inside the lane's run
// [off0, off0 + np)
__device__ __forceinline__ uint32_t matched_mask16(int4 c0, int4 c1, int4 c2, int4 c3, uint32_t g0,
                                                   uint32_t off0, uint32_t np) {
    const int32_t v[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                           c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) m |= (uint32_t)(v[j] >= 0) << j;
    if (g0 < off0) m &= 0xffffu << off0;
    if (g0 + 16u > off0 + np) m &= (1u << (off0 + np - g0)) - 1u;
    return m;
}

// bit j: entry g0 + j of an aligned 8-entry pend[] group is a match (>= 0) inside the lane's run
// [off0, off0 + np)
__device__ __forceinline__ uint32_t matched_mask8(int4 c0, int4 c1, uint32_t g0, uint32_t off0, uint32_t np) {
    const int32_t v[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) m |= (uint32_t)(v[j] >= 0) << j;
    if (g0 < off0) m &= 0xffu << off0;
    if (g0 + 8u > off0 + np) m &= (1u << (off0 + np - g0)) - 1u;
    return m;
}

// Per scan lane: its pairs in (utterance, start, accept-set) order.  Unmatched pairs change no state
// (finditer skipping, exclusion and overlap only see matches), so only matched ones are decoded.
// Findings go to the LANE's arena (fd + fd_base), in (utterance, start) order; lane_nf counts them.
// A whole utterance's output length is written directly; a cut row's findings are split over its
// lanes, whose deltas (token length - match length) k_rowlen adds up.  A lane that continues a cut
// row starts with a fresh state, which is exact unless a match of the previous lanes reaches into it
// (lane_reach); k_sel_dirty / k_sel_fix re-run those lanes with the carried state.
struct SelTabs {
    const uint16_t* dtype;
    const uint8_t* ven;
    const uint8_t* vmin;
    const uint8_t* dex;
    const void* xix;          // exclusion lists (list_range)
    uint32_t xw;
    const uint32_t* xloff;
    const uint16_t* xids;
    const uint32_t* tokoff;
};
struct SelIO {
    const uint64_t* lane_pair;
    const uint32_t* lane_np;
    const SelRec* sel;
    const int32_t* pend;
    uint64_t pair_cap;
    const uint8_t* role;
    const int16_t* ctx;
    pii_span* fd;
    uint32_t* lane_nf;
    int2* lane_rd;          // cut-row deltas: .x = row u0 (lane cut at lo), .y = row u1 - 1 (cut at hi)
    uint32_t* lane_reach;   // lanes cut at hi: furthest match end of the cut row (row relative)
    uint32_t* out_len;
    uint2* spill;           // per pair-queue index: the (pattern, end) list of a run past LIVE patterns
    // external candidates (another detector's spans, e.g. the NER's PERSON_NAME): ext[row * ext_stride
    // + k] for k < ext_n[row], row-relative, sorted by start; only read by select_run<true>
    const pii_span* ext;
    const uint32_t* ext_n;
    uint32_t ext_stride;
    uint32_t* err;          // ERR_EXT: a malformed external span
    // the per-(variant, type) exclusion lists in global memory (L2) when the LDS image omits them
    // (config 5's are 93 KB: with them k_select held one 256-thread workgroup per CU); else null
    const uint32_t* g_xoff;
    const uint16_t* g_xids;
};

__device__ __forceinline__ uint64_t fd_base(const Lane& L, uint32_t c, int min_len) {
    return (uint64_t)(L.lo / (uint32_t)min_len) + c;
}

__device__ __forceinline__ SelTabs sel_tabs(const uint8_t* lb, const LdsImage& li) {
    SelTabs T;
    T.dtype = reinterpret_cast<const uint16_t*>(lb + li.off[SE_DTYPE]);
    T.ven = lb + li.off[SE_VEN];
    T.vmin = lb + li.off[SE_VMIN];
    T.dex = lb + li.off[SE_DEX];
    T.xix = lb + li.off[SE_XOFF];
    T.xw = (li.aux >> 3) & 7u;
    T.xloff = reinterpret_cast<const uint32_t*>(lb + li.off[SE_XLOFF]);
    T.xids = reinterpret_cast<const uint16_t*>(lb + li.off[SE_XIDS]);
    T.tokoff = reinterpret_cast<const uint32_t*>(lb + li.off[SE_TOKOFF]);
    return T;
}

// The selection state machine of ONE pass over candidates in (row, start, accept-set) order: finditer
// skipping per pattern, exclusion (A.5), best-per-start and greedy overlap resolution (A.6), output
// sizing.  Findings go to the current LANE's arena (fd + fd_base), in (utterance, start) order.  Fed
// by select_run (k_select / k_sel_fix: candidates from the global pair queue).
struct LaneSel {
    // per-utterance state
    uint32_t u;
    int v, minlik;
    int lp[LIVE], le[LIVE];
    uint32_t n_spill;
    bool spilled;
    int ex_s[NE_MAX], ex_e[NE_MAX], ex_t[NE_MAX];
    uint32_t ex_valid;
    int max_end;
    uint32_t nf_u;
    int delta_u;
    // per-lane state
    Lane Lg;
    pii_span* fdl;
    uint32_t nfl;
    int rdx, rdy;
    uint32_t reach;
    // per-start state
    int s, best_e, best_t, best_lik;
    uint2* spill;           // the lane run's list of (pattern, end) once more than LIVE patterns are live

    __device__ __forceinline__ void init(uint2* sp) {
        spill = sp;
        u = 0xffffffffu;
        v = 0;
        minlik = 0;
        n_spill = 0;
        spilled = false;
        ex_valid = 0;
        max_end = 0;
        nf_u = 0;
        delta_u = 0;
        Lg = Lane{};
        fdl = nullptr;
        nfl = 0;
        rdx = rdy = 0;
        reach = 0;
        s = -1;
        best_e = -1;
        best_t = 0;
        best_lik = 0;
#pragma unroll
        for (int q = 0; q < LIVE; ++q) {
            lp[q] = -1;
            le[q] = -1;
        }
#pragma unroll
        for (int x = 0; x < NE_MAX; ++x) ex_s[x] = ex_e[x] = ex_t[x] = 0;
    }
    __device__ __forceinline__ bool cut_lo_row(uint32_t x) const { return Lg.clo && x == Lg.u0; }
    __device__ __forceinline__ bool cut_row(uint32_t x) const { return cut_lo_row(x) || (Lg.chi && x == Lg.u1 - 1); }
    // a new lane of the pass: its findings arena and per-lane outputs start empty
    __device__ __forceinline__ void begin_lane(const Geo& g, const SelIO& io, const RulesDev& R, uint32_t lane) {
        Lg = g_lane(g, lane);
        fdl = io.fd + fd_base(Lg, lane, R.min_len);
        nfl = 0;
        rdx = rdy = 0;
        reach = 0;
    }
    __device__ __forceinline__ void flush_start(const SelTabs& Tb) {
        if (best_e >= 0 && s >= max_end) {
            pii_span f;
            f.utt = u;
            f.start = (uint32_t)s;
            f.end = (uint32_t)best_e;
            f.info_type = (uint16_t)best_t;
            f.likelihood = (uint8_t)best_lik;
            f.flags = 0;
            fdl[nfl++] = f;
            max_end = best_e;
            const int d = (int)(Tb.tokoff[best_t + 1] - Tb.tokoff[best_t]) - (best_e - s);
            // (selects, not branches: a branch on which counter to add to makes the compiler keep
            // the counters in a scratch array)
            const bool clo_r = cut_lo_row(u), cut_r = cut_row(u);
            rdx += clo_r ? d : 0;
            rdy += (cut_r && !clo_r) ? d : 0;
            delta_u += cut_r ? 0 : d;
            nf_u += cut_r ? 0u : 1u;
        }
        best_e = -1;
    }
    // a whole row's output length, written (not added: k_sel_fix re-runs whole lanes, and a re-run
    // must not count the whole rows of its lanes twice); rows without findings keep the length
    // k_chunk_index wrote
    __device__ __forceinline__ void flush_utt(const Geo& g, const SelIO& io) {
        if (nf_u) io.out_len[u] = (uint32_t)(g_off(g, u + 1) - g_off(g, u)) + (uint32_t)delta_u;
    }
    // candidate (row pu, start ps, end e) enters: row / start transitions
    // pv: the row's context variant, or -1: derive it from role / ctx
    __device__ __forceinline__ void enter(const SelTabs& Tb, const Geo& g, const SelIO& io, uint32_t pu, int ps, int e,
                                          int pv) {
        if (pu != u) {
            if (u != 0xffffffffu) {
                flush_start(Tb);
                flush_utt(g, io);
            }
            u = pu;
            v = pv >= 0 ? pv : (io.role[u] == PII_ROLE_CUSTOMER && io.ctx[u] >= 0) ? io.ctx[u] + 1 : 0;
            minlik = Tb.vmin[v];
#pragma unroll
            for (int q = 0; q < LIVE; ++q) {
                lp[q] = -1;
                le[q] = -1;
            }
            spilled = false;
            n_spill = 0;
            ex_valid = 0;
            max_end = 0;
            nf_u = 0;
            delta_u = 0;
            s = ps;
        } else if (ps != s) {
            flush_start(Tb);
            s = ps;
        }
        if (Lg.chi && u == Lg.u1 - 1) reach = max(reach, (uint32_t)e);
    }
    // a valid candidate of type t (excluder slot xi, 0xff: none) competes for its start
    template <bool CL>
    __device__ __forceinline__ void consider(const SelTabs& Tb, int T, int t, int lik, int e, int xi) {
        uint32_t x0, x1;
        list_range<CL>(Tb.xix, Tb.xw, Tb.xloff, (uint32_t)(v * T + t), x0, x1);
        bool excluded = false;
        for (uint32_t q = x0; q < x1; ++q) {
            const int xt = Tb.xids[q];
#pragma unroll
            for (int x = 0; x < NE_MAX; ++x)
                if (x != xi && ((ex_valid >> x) & 1) && ex_t[x] == xt && ex_s[x] <= s && e <= ex_e[x])
                    excluded = true;
        }
        if (excluded) return;
        const bool better = best_e < 0 || e > best_e ||
                            (e == best_e && (lik > best_lik || (lik == best_lik && t < best_t)));
        if (better) {
            best_e = e;
            best_t = t;
            best_lik = lik;
        }
    }
    // a matched pair: row pu, start ps (row relative), pattern p, context variant pv, end e, likelihood lik
    template <bool CL>
    __device__ __forceinline__ void pair(const SelTabs& Tb, const Geo& g, const SelIO& io, int T, uint32_t pu, int ps,
                                         int p, int pv, int e, int lik) {
        enter(Tb, g, io, pu, ps, e, pv);
        const int t = Tb.dtype[p];
        if (!Tb.ven[v * T + t]) return;
        int prev_end = -1;
        if (spilled) {
            for (uint32_t q = 0; q < n_spill; ++q)
                if ((int)spill[q].x == p) prev_end = (int)spill[q].y;
        } else {
#pragma unroll
            for (int q = 0; q < LIVE; ++q)
                if (lp[q] == p) prev_end = le[q];
        }
        if (s < prev_end) return;               // inside p's previous match (finditer)
        if (spilled) {
            uint32_t q = 0;
            while (q < n_spill && (int)spill[q].x != p) ++q;
            spill[q] = make_uint2((uint32_t)p, (uint32_t)e);
            if (q == n_spill) ++n_spill;
        } else {
            int slot = -1;
#pragma unroll
            for (int q = 0; q < LIVE; ++q)
                if (lp[q] == p) slot = q;
            if (slot < 0) {
#pragma unroll
                for (int q = 0; q < LIVE; ++q)
                    if (slot < 0 && le[q] <= s) slot = q;
            }
            if (slot >= 0) {
#pragma unroll
                for (int q = 0; q < LIVE; ++q)
                    if (q == slot) {
                        lp[q] = p;
                        le[q] = e;
                    }
            } else {                             // more than LIVE patterns live: list in global memory
                n_spill = 0;
#pragma unroll
                for (int q = 0; q < LIVE; ++q)
                    if (lp[q] >= 0) spill[n_spill++] = make_uint2((uint32_t)lp[q], (uint32_t)le[q]);
                spill[n_spill++] = make_uint2((uint32_t)p, (uint32_t)e);
                spilled = true;
            }
        }
        const int xi = Tb.dex[p];
        if (lik < minlik) {                        // invalid (-1) or below min_likelihood
            if (xi != 0xff) ex_valid &= ~(1u << xi);
            return;
        }
        if (xi != 0xff) {
#pragma unroll
            for (int x = 0; x < NE_MAX; ++x)
                if (x == xi) {
                    ex_s[x] = s;
                    ex_e[x] = e;
                    ex_t[x] = t;
                }
            ex_valid |= 1u << xi;
        }
        consider<CL>(Tb, T, t, lik, e, xi);
    }
    // the end of the lane: the pending start and (unless the row continues into the next lane) the
    // utterance end; the lane's outputs
    __device__ __forceinline__ void end_lane(const SelTabs& Tb, const Geo& g, const SelIO& io, uint32_t lane) {
        if (u != 0xffffffffu) {
            flush_start(Tb);
            if (!(Lg.chi && u == Lg.u1 - 1)) {
                flush_utt(g, io);
                u = 0xffffffffu;
            }
        }
        io.lane_nf[lane] = nfl;
        io.lane_rd[lane] = make_int2(rdx, rdy);
        if (Lg.chi) io.lane_reach[lane] = reach;
    }
};

// select over the pairs of lanes c0..c1 as ONE sequential pass (the state carries across the lanes).
// EXT: the lanes' external candidates (SelIO::ext) are merged into the pair stream in (row, start)
// order; they take part in overlap resolution (A.6) and min_likelihood like any finding, but not in
// finditer skipping (they have no pattern) nor as excluders.
template <bool EXT, bool CL>
__device__ void select_run(const RulesDev& R, const SelTabs& Tb, const Geo& g, const SelIO& io, uint32_t c0,
                           uint32_t c1) {
    const int T = R.T;
    LaneSel S;
    S.init(io.spill + io.lane_pair[c0]);
    // external candidates: cursor over the lane's rows [u0, u1); a cut row contributes the spans
    // whose start lies in the lane's byte range.  Every span is checked (start < end <= row length,
    // sorted by start, type < T, likelihood 1..5); a bad one sets ERR_EXT and is skipped.
    uint32_t xu = 0, xk = 0, xn = 0, xprev = 0;
    pii_span X{};
    bool xhave = false;
    auto xrow = [&](uint32_t r) {
        xu = r;
        xk = 0;
        xprev = 0;
        xn = 0;
        if (r < S.Lg.u1) {
            xn = io.ext_n[r];
            if (xn > io.ext_stride) {
                atomicOr(io.err, ERR_EXT);
                xn = io.ext_stride;
            }
        }
    };
    auto xload = [&]() {
        xhave = false;
        while (xu < S.Lg.u1) {
            if (xk < xn) {
                X = io.ext[(uint64_t)xu * io.ext_stride + xk++];
                const int64_t r0 = g_off(g, xu), rl = g_off(g, xu + 1) - r0;
                if (X.end <= X.start || (int64_t)X.end > rl || X.start < xprev || (int)X.info_type >= T ||
                    X.likelihood == 0 || X.likelihood > 5) {
                    atomicOr(io.err, ERR_EXT);
                    continue;
                }
                xprev = X.start;
                const int64_t a = r0 + X.start;
                if (S.Lg.clo && xu == S.Lg.u0 && a < (int64_t)S.Lg.lo) continue;
                if (S.Lg.chi && xu == S.Lg.u1 - 1 && a >= (int64_t)S.Lg.hi) {
                    xk = xn;
                    continue;
                }
                X.utt = xu;
                xhave = true;
                return;
            }
            xrow(xu + 1);
        }
    };
    auto ext_cand = [&]() {
        const int e = (int)X.end, t = X.info_type, lik = X.likelihood;
        S.enter(Tb, g, io, X.utt, (int)X.start, e, -1);
        if (Tb.ven[S.v * T + t] && lik >= S.minlik) S.template consider<CL>(Tb, T, t, lik, e, 0xff);
        xload();
    };
    for (uint32_t lane = c0; lane <= c1; ++lane) {
        S.begin_lane(g, io, R, lane);
        if (EXT) {
            xrow(S.Lg.u0);
            xload();
        }
        const uint32_t np = io.lane_np[lane];
        const uint64_t pbase = io.lane_pair[lane];
        if (np && pbase + np <= io.pair_cap) {
            // pend[] (4 B per pair, the lane's run) is read 8 entries per iteration as two aligned
            // 16-byte loads, the next group issued before this one is decoded; only matched pairs
            // (e >= 0, a small fraction) enter the body.  pend is allocated 16 entries past pair_cap,
            // so the aligned groups never leave the allocation; entries outside the run are masked off.
            // (8, not 16, entries per group, LIVE = 5 and NE_MAX = 2 keep k_select at 5 waves/SIMD)
            const int32_t* el = io.pend + pbase;
            const uint32_t off0 = (uint32_t)(pbase & 3u);
            const int4* pa = reinterpret_cast<const int4*>(io.pend + (pbase - off0));
            const uint32_t ng = (off0 + np + 7u) >> 3;
            int4 q0 = pa[0], q1 = pa[1];
            uint32_t gi = 0, g0 = 0, m = 0;
            // the next matched pair of the run (false: none left)
            auto adv = [&](uint32_t& i) -> bool {
                while (m == 0) {
                    if (gi >= ng) return false;
                    const int4 d0 = q0, d1 = q1;
                    if (gi + 1 < ng) {
                        const int4* pn = pa + 2 * (gi + 1);
                        q0 = pn[0];
                        q1 = pn[1];
                    }
                    g0 = 8u * gi;
                    m = matched_mask8(d0, d1, g0, off0, np);
                    ++gi;
                }
                const uint32_t j = (uint32_t)__builtin_ctz(m);
                m &= m - 1u;
                i = g0 + j - off0;
                return true;
            };
            // each matched pair's SelRec is loaded one pair ahead of its use
            uint32_t i1 = 0;
            bool ok = adv(i1);
            SelRec r1{};
            if (ok) r1 = io.sel[pbase + i1];
            while (ok) {
                const SelRec r = r1;
                const int e = el[i1];          // (in L1: its group was just loaded)
                ok = adv(i1);
                if (ok) r1 = io.sel[pbase + i1];
                if (EXT)
                    while (xhave && (X.utt < r.u || (X.utt == r.u && (int)X.start <= r.ps))) ext_cand();
                S.template pair<CL>(Tb, g, io, T, r.u, r.ps, (int)(r.p & 0xffffu), (int)(r.p >> 16), e, r.lik);
            }
        }
        if (EXT)
            while (xhave) ext_cand();
        S.end_lane(Tb, g, io, lane);
    }
}

template <bool GI, bool EXT, bool CL = false>
__global__ __launch_bounds__(256) void k_select(const RulesDev R, const uint4* __restrict__ img, const LdsImage li,
                                                const Geo g, const SelIO io, const uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    if (*err & ERR_ABORT) return;           // the batch is re-run with a larger queue
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    SelTabs Tb = sel_tabs(lb, li);
    if (io.g_xoff) {
        Tb.xix = nullptr;
        Tb.xw = 0;
        Tb.xloff = io.g_xoff;
        Tb.xids = io.g_xids;
    }
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= g.n_chunks) return;
    select_run<EXT, CL>(R, Tb, g, io, c, c);
}

// ---- cut rows: which continuation lanes need the carried state (a match of an earlier lane of the
// row reaches past their first start), one workgroup per long row.  dirty[c] is written for every
// lane of the row (0 for the lane holding the row start unless it continues another cut row).
constexpr int ROW_BLOCK = 1024;

// inclusive max / sum scans over a row's lanes, ROW_BLOCK x 4 per round
__device__ __forceinline__ uint32_t block_incl_max(uint32_t x, uint32_t* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(x, d);
        if (lane >= d) x = max(x, o);
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wid; ++w) pre = max(pre, sh[w]);
    __syncthreads();
    return max(x, pre);
}

__global__ __launch_bounds__(ROW_BLOCK) void k_sel_dirty(const Geo g, const uint32_t* __restrict__ long_rows,
                                                        const uint32_t* __restrict__ long_count,
                                                        const uint32_t* __restrict__ lane_reach,
                                                        uint8_t* __restrict__ dirty, const uint32_t* __restrict__ err) {
    __shared__ uint32_t sh[ROW_BLOCK / 64];
    __shared__ uint32_t s_carry;
    if (*err & (ERR_ABORT | ERR_STITCH)) return;
    for (uint32_t ri = blockIdx.x; ri < *long_count; ri += gridDim.x) {
        uint32_t ca, kb;
        int64_t s_r, e_r;
        row_lanes(g, long_rows[ri], ca, kb, s_r, e_r);
        if (threadIdx.x == 0) {
            s_carry = 0;
            if (!g_cut(g, ca)) dirty[ca] = 0;
        }
        __syncthreads();
        // dirty[c] (c in (ca, kb]) = max(reach over lanes [ca, c)) > first start of c (row relative)
        for (uint32_t c0 = ca; c0 < kb; c0 += ROW_BLOCK) {
            const uint32_t j = c0 + threadIdx.x;        // lane j's reach feeds dirty[j + 1]
            const uint32_t x = j < kb ? lane_reach[j] : 0u;
            const uint32_t incl = max(block_incl_max(x, sh), s_carry);
            if (j < kb) {
                const int64_t first = g_cpos(g, j + 1) + 1 - s_r;
                dirty[j + 1] = (int64_t)incl > first ? 1 : 0;
            }
            __syncthreads();
            if (threadIdx.x == ROW_BLOCK - 1) s_carry = incl;
            __syncthreads();
        }
    }
}

// re-run every maximal chain of dirty lanes from the clean lane before it (one thread per chain)
template <bool GI, bool EXT, bool CL = false>
__global__ __launch_bounds__(256) void k_sel_fix(const RulesDev R, const uint4* __restrict__ img, const LdsImage li,
                                                 const Geo g, const SelIO io, const uint32_t* __restrict__ long_rows,
                                                 const uint32_t* __restrict__ long_count,
                                                 const uint8_t* __restrict__ dirty, const uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    if ((*err & (ERR_ABORT | ERR_STITCH)) || blockIdx.x >= *long_count) return;     // (before the image load)
    // the row's chain starts are compacted first, so the chains run side by side (a thread per lane
    // left most threads idle and ran the few chains of a row one slice of 256 lanes after another)
    constexpr uint32_t FIX_CAP = 256;
    static_assert(FIX_CAP >= 256, "a slice of the launch's 256 lanes always fits an emptied list");
    __shared__ uint32_t s_chain[FIX_CAP];
    __shared__ uint32_t s_wc[4];
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    SelTabs Tb = sel_tabs(lb, li);
    if (io.g_xoff) {
        Tb.xix = nullptr;
        Tb.xw = 0;
        Tb.xloff = io.g_xoff;
        Tb.xids = io.g_xids;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t ri = blockIdx.x; ri < *long_count; ri += gridDim.x) {
        uint32_t ca, kb;
        int64_t s_r, e_r;
        row_lanes(g, long_rows[ri], ca, kb, s_r, e_r);
        // chain starts listed in lane order one slice of 256 lanes at a time; the listed chains run
        // when the next slice might not fit and after the last one -- ONE call site of select_run, so
        // it is inlined (two sites kept it a call: 180 VGPRs and 560 B of scratch per lane)
        uint32_t n = 0;                                   // chains listed (block-uniform)
        for (uint32_t j0 = ca;; j0 += 256) {
            const bool done = j0 >= kb;
            const uint32_t j = j0 + threadIdx.x;
            const bool st = !done && j < kb && !dirty[j] && dirty[j + 1];
            const uint32_t tot = (uint32_t)__syncthreads_count(st);
            if (done || n + tot > FIX_CAP) {
                for (uint32_t k = threadIdx.x; k < n; k += 256) {
                    const uint32_t j1 = s_chain[k];
                    uint32_t c = j1 + 1;
                    while (c + 1 < g.n_chunks && g_cut(g, c + 1) && dirty[c + 1]) ++c;
                    select_run<EXT, CL>(R, Tb, g, io, j1, c);
                }
                n = 0;
                __syncthreads();                          // the list is free again
            }
            if (done) break;
            const uint64_t bal = __ballot(st);
            if (lane == 0) s_wc[wv] = (uint32_t)__popcll(bal);
            __syncthreads();
            uint32_t pre = n;
            for (int w = 0; w < wv; ++w) pre += s_wc[w];
            if (st) s_chain[pre + __popcll(bal & ((1ull << lane) - 1))] = j;
            n += tot;
            __syncthreads();                              // (s_wc is reused by the next slice)
        }
    }
}

// a cut row's output length (its lanes' deltas) and, per continuation lane, the delta of the row's
// findings in the lanes before it (k_spans places the row's findings in the output with it)
__global__ __launch_bounds__(ROW_BLOCK) void k_rowlen(const Geo g, const uint32_t* __restrict__ long_rows,
                                                     const uint32_t* __restrict__ long_count,
                                                     const int2* __restrict__ lane_rd, int32_t* __restrict__ lane_rowbase,
                                                     uint32_t* __restrict__ out_len, const uint32_t* __restrict__ err) {
    __shared__ int32_t sh[ROW_BLOCK / 64];
    __shared__ int32_t s_carry;
    if (*err & (ERR_ABORT | ERR_STITCH)) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t ri = blockIdx.x; ri < *long_count; ri += gridDim.x) {
        const uint32_t r = long_rows[ri];
        uint32_t ca, kb;
        int64_t s_r, e_r;
        row_lanes(g, r, ca, kb, s_r, e_r);
        if (threadIdx.x == 0) s_carry = 0;
        __syncthreads();
        for (uint32_t c0 = ca; c0 <= kb; c0 += ROW_BLOCK) {
            const uint32_t c = c0 + threadIdx.x;
            int32_t x = 0;
            if (c <= kb) x = c == ca ? lane_rd[c].y : lane_rd[c].x;
            int32_t incl = x;
            for (int d = 1; d < 64; d <<= 1) {
                const int32_t o = __shfl_up(incl, d);
                if (lane >= d) incl += o;
            }
            if (lane == 63) sh[wid] = incl;
            __syncthreads();
            int32_t pre = s_carry;
            for (int w = 0; w < wid; ++w) pre += sh[w];
            if (c <= kb && c > ca) lane_rowbase[c] = pre + incl - x;
            __syncthreads();
            if (threadIdx.x == ROW_BLOCK - 1) s_carry = pre + incl;
            __syncthreads();
        }
        if (threadIdx.x == 0) out_len[r] = (uint32_t)((e_r - s_r) + s_carry);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------- exclusive scans
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(x, d);
        if (lane >= d) x += o;
    }
    return x;
}

// block-level exclusive scan of 256 threads x SCAN_ITEMS; returns block total
__device__ uint64_t block_exscan(uint64_t (&v)[SCAN_ITEMS], uint64_t* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t tsum = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t x = v[i];
        v[i] = tsum;
        tsum += x;
    }
    const uint64_t inc = wave_incl_scan(tsum, lane);
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    uint64_t wpre = 0, total = 0;
    for (int w = 0; w < 4; ++w) {
        if (w < wid) wpre += sh[w];
        total += sh[w];
    }
    const uint64_t tpre = wpre + inc - tsum;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) v[i] += tpre;
    __syncthreads();
    return total;
}

// Up to two independent scans per launch (blockIdx.y picks one: the two per-lane scans of the front go
// together); a thread owns SCAN_ITEMS consecutive entries, read / written with 16-byte accesses when
// the arrays allow it.
struct ScanArgs {
    const uint32_t* in[2];
    uint64_t* out[2];
    uint32_t n[2];
    uint32_t bstride;            // block sums of scan 1 at bsum + bstride
};

__device__ __forceinline__ void scan_load(const uint32_t* __restrict__ in, uint32_t n, uint64_t i0,
                                          uint32_t (&v)[SCAN_ITEMS]) {
    if (i0 + SCAN_ITEMS <= n && ((uintptr_t)(in + i0) & 15) == 0) {
        const uint4 a = *reinterpret_cast<const uint4*>(in + i0), b = *reinterpret_cast<const uint4*>(in + i0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) v[i] = i0 + i < n ? in[i0 + i] : 0u;
    }
}

__global__ __launch_bounds__(256) void k_scan_reduce(const ScanArgs a, uint64_t* __restrict__ bsum) {
    __shared__ uint64_t sh[4];
    const int y = blockIdx.y;
    const uint32_t n = a.n[y];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    if (base >= n && blockIdx.x > 0) return;
    uint32_t v[SCAN_ITEMS];
    scan_load(a.in[y], n, base + (uint64_t)threadIdx.x * SCAN_ITEMS, v);
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) s += v[i];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    s = wave_incl_scan(s, lane);
    if (lane == 63) sh[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[y * a.bstride + blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// one workgroup per scan: exclusive scan of its block sums in place (serial over tiles)
__global__ __launch_bounds__(256) void k_scan_blocks(const ScanArgs a, uint64_t* __restrict__ bsum0) {
    __shared__ uint64_t sh[4];
    const int y = blockIdx.x;
    uint64_t* __restrict__ bsum = bsum0 + y * a.bstride;
    const uint32_t nb = (a.n[y] + SCAN_TILE - 1) / SCAN_TILE;
    uint64_t carry = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += SCAN_TILE) {
        uint64_t v[SCAN_ITEMS];
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const uint32_t idx = c0 + threadIdx.x * SCAN_ITEMS + i;
            v[i] = idx < nb ? bsum[idx] : 0;
        }
        const uint64_t tot = block_exscan(v, sh);
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const uint32_t idx = c0 + threadIdx.x * SCAN_ITEMS + i;
            if (idx < nb) bsum[idx] = v[i] + carry;
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

// out[i] = exclusive prefix of in[]; out[n] = total
__global__ __launch_bounds__(256) void k_scan_apply(const ScanArgs a, const uint64_t* __restrict__ bsum) {
    __shared__ uint64_t sh[4];
    const int y = blockIdx.y;
    const uint32_t n = a.n[y];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    if (base >= n) {
        if (base == 0 && threadIdx.x == 0) a.out[y][0] = 0;
        return;
    }
    const uint32_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
    const uint64_t i0 = base + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t x[SCAN_ITEMS];
    scan_load(a.in[y], n, i0, x);
    uint64_t v[SCAN_ITEMS];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) v[i] = x[i];
    block_exscan(v, sh);
    const uint64_t off = bsum[y * a.bstride + blockIdx.x];
    uint64_t* __restrict__ out = a.out[y];
    if (i0 + SCAN_ITEMS <= n && ((uintptr_t)(out + i0) & 15) == 0) {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; i += 2)
            *reinterpret_cast<ulonglong2*>(out + i0 + i) = make_ulonglong2(v[i] + off, v[i + 1] + off);
    } else {
        for (int i = 0; i < SCAN_ITEMS; ++i)
            if (i0 + i < n) out[i0 + i] = v[i] + off;
    }
    if (blockIdx.x == nt - 1 && threadIdx.x == 0) out[n] = bsum[y * a.bstride + nt];
}

// Single-pass exclusive scan (decoupled look-back): out[i] = in[0] + ... + in[i-1], out[n] = total.
// A workgroup takes the next tile by ticket (so it only ever waits on tiles that are already running),
// publishes its aggregate, then walks back over predecessors' published words until an inclusive
// prefix.  A tile word is one 64-bit atomic: [epoch:24][status:2][value:38]; the epoch tells this
// launch's words from stale ones, so the state array is never cleared.  ctr[0] = ticket counter,
// ctr[1] = finished workgroups: the last one to finish zeroes both for the next launch.
constexpr int LB_BLOCK = 256, LB_ITEMS = 16, LB_TILE = LB_BLOCK * LB_ITEMS;
constexpr uint64_t LB_AGG = 1, LB_INCL = 2;

__device__ __forceinline__ uint64_t lb_word(uint32_t epoch, uint64_t status, uint64_t v) {
    return ((uint64_t)(epoch & 0xffffffu) << 40) | (status << 38) | (v & ((1ull << 38) - 1));
}

// up to two independent scans in one launch (blockIdx.y: its own input, tiles, tile states and
// ticket pair); a block whose ticket is past its scan's tiles only counts itself out
struct LbArgs {
    const uint32_t* in[2];
    uint64_t* out[2];
    uint32_t n[2], nb[2];
    uint32_t sstride;        // tile-state words per scan
};

__global__ __launch_bounds__(LB_BLOCK) void k_scan_lb(const LbArgs a, unsigned long long* state0,
                                                      unsigned long long* ctr0, uint32_t epoch) {
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_prefix;
    __shared__ uint64_t s_w[LB_BLOCK / 64];
    const uint32_t y = blockIdx.y;
    const uint32_t* __restrict__ in = a.in[y];
    uint64_t* __restrict__ out = a.out[y];
    const uint32_t n = a.n[y], nbt = a.nb[y];
    unsigned long long* state = state0 + (size_t)y * a.sstride;
    unsigned long long* ctr = ctr0 + 2 * y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) s_tile = (uint32_t)atomicAdd(&ctr[0], 1ull);
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= nbt) {
        if (tid == 0 && atomicAdd(&ctr[1], 1ull) == gridDim.x - 1) {
            ctr[0] = 0;
            ctr[1] = 0;
        }
        return;
    }
    const uint64_t i0 = (uint64_t)tile * LB_TILE + (uint64_t)tid * LB_ITEMS;
    uint32_t v[LB_ITEMS];
    if (i0 + LB_ITEMS <= n && ((uintptr_t)(in + i0) & 15) == 0) {
        const uint4* p = reinterpret_cast<const uint4*>(in + i0);
#pragma unroll
        for (int k = 0; k < LB_ITEMS / 4; ++k) {
            const uint4 x = p[k];
            v[4 * k] = x.x;
            v[4 * k + 1] = x.y;
            v[4 * k + 2] = x.z;
            v[4 * k + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < LB_ITEMS; ++k) v[k] = i0 + k < n ? in[i0 + k] : 0u;
    }
    uint64_t tsum = 0;
#pragma unroll
    for (int k = 0; k < LB_ITEMS; ++k) tsum += v[k];
    uint64_t incl = tsum;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint64_t wpre = 0, total = 0;
    for (int w = 0; w < LB_BLOCK / 64; ++w) {
        if (w < wid) wpre += s_w[w];
        total += s_w[w];
    }
    if (wid == 0) {
        // wavefront 0: publish, then look back 64 predecessors at a time (one word per lane)
        uint64_t prefix = 0;
        if (tile == 0) {
            if (lane == 0)
                __hip_atomic_store(&state[0], lb_word(epoch, LB_INCL, total), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&state[tile], lb_word(epoch, LB_AGG, total), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            int64_t top = (int64_t)tile - 1;               // nearest predecessor of this window
            for (;;) {
                const int64_t j = top - lane;
                uint64_t w = 0, st = LB_INCL, val = 0;     // lanes past tile 0 act as a zero inclusive word
                if (j >= 0) {
                    w = __hip_atomic_load(&state[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    st = ((uint32_t)(w >> 40) == (epoch & 0xffffffu)) ? (w >> 38) & 3 : 0;
                    val = w & ((1ull << 38) - 1);
                }
                const uint64_t incl_mask = __ballot(st == LB_INCL);
                const uint64_t ready = __ballot(st != 0);
                // the nearest inclusive word ends the walk; every word before it must be ready
                const int stop = incl_mask ? __builtin_ctzll(incl_mask) : 64;
                const uint64_t need = stop == 64 ? ~0ull : ((2ull << stop) - 1);
                if ((ready & need) != need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint64_t x = lane <= stop ? val : 0;
                for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
                prefix += x;
                if (stop < 64) break;
                top -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&state[tile], lb_word(epoch, LB_INCL, prefix + total), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_prefix = prefix;
    }
    __syncthreads();
    uint64_t run = s_prefix + wpre + incl - tsum;
    if (i0 + LB_ITEMS <= n) {
#pragma unroll
        for (int k = 0; k < LB_ITEMS; ++k) {
            out[i0 + k] = run;
            run += v[k];
        }
    } else {
        for (int k = 0; k < LB_ITEMS; ++k) {
            if (i0 + k < n) out[i0 + k] = run;
            run += v[k];
        }
    }
    if (tile == nbt - 1 && tid == 0) out[n] = s_prefix + total;
    if (tid == 0 && atomicAdd(&ctr[1], 1ull) == gridDim.x - 1) {
        ctr[0] = 0;
        ctr[1] = 0;
    }
}

__global__ void k_finalize(const uint64_t* __restrict__ out_offs, const uint64_t* __restrict__ span_offs,
                           uint32_t n_utt, uint32_t n_span_rows, uint64_t out_cap, uint64_t span_cap, uint32_t* __restrict__ err,
                           uint64_t* __restrict__ totals, const unsigned long long* __restrict__ pair_count,
                           const uint64_t* __restrict__ ev_count, const uint64_t* __restrict__ wf_count) {
    const uint64_t ob = out_offs[n_utt], ns = span_offs[n_span_rows];
    if (ob > out_cap || ns > span_cap) atomicOr(err, (uint32_t)ERR_CAPACITY);
    totals[0] = ob;
    totals[1] = ns;
    totals[2] = *err;
    totals[3] = *pair_count;
    totals[4] = ev_count ? *ev_count : 0;
    totals[5] = wf_count ? *wf_count : 0;
}

// ---------------------------------------------------------------------------------- k_redact
// Span-driven scatter.  Utterance boundaries do not matter to the copy: the output is the batch's
// bytes with every kept span replaced by its "[INFO_TYPE]" token, i.e. long copy runs (~1 KiB apart at
// config 2) and short tokens.  k_spans lists every span with its input range and output position
// (RSpan, in batch order); a workgroup then owns one 64 KiB tile of the OUTPUT (address-aligned),
// finds its first span (k_tile_first), builds the tile's PIECE table in LDS (copy runs and tokens)
// and a block -> piece table, and lane i assembles aligned 16-byte output blocks i, i+256, ... so
// every load and store instruction of a wavefront covers 1 KiB of consecutive bytes: a block inside
// one piece is two aligned 16-byte source loads + a funnel shift (v_alignbyte), a block that
// straddles pieces ORs the masked windows of each piece it touches.  Source bytes never pass through
// LDS.  A tile with more spans than the piece table holds is assembled in several passes.  Rows of
// any length (a whole transcript) take the same path.
#ifndef REDACT_BLOCK_N
#define REDACT_BLOCK_N 256
#endif
constexpr int REDACT_BLOCK = REDACT_BLOCK_N;
#ifndef REDACT_ABLATE
#define REDACT_ABLATE 0             // measurement builds only: 1 = no assembly, 2 = tables only, 3 = no source loads
#endif
#ifndef REDACT_NT
#define REDACT_NT 1                 // non-temporal output stores in the pipelined loop
#endif
#ifndef REDACT_PIPE
#define REDACT_PIPE 1               // tile_assemble's pipelined interior-block loop (0: one block at a time)
#endif
constexpr int PIECE_MAX = 1024;
#ifndef RTILE_SHIFT_N
#define RTILE_SHIFT_N 16
#endif
constexpr uint32_t RTILE_SHIFT = RTILE_SHIFT_N;  // output tile: 64 KiB = BLK_MAX blocks
constexpr int BLK_MAX = 1 << (RTILE_SHIFT - 4);  // output blocks covered by the block -> piece table
constexpr int SPAN_PASS = REDACT_BLOCK - 1;   // spans per assembly pass: one per thread (2 pieces each + 2 <= PIECE_MAX)

struct RSpan {          // one kept span in batch order (16 B)
    uint64_t out;       // output position of its token | info type << 48
    uint32_t in_lo;     // input range [in_lo, in_hi), batch relative
    uint32_t in_hi;
};

// Output assembly shared by k_redact and k_win_redact.  The piece table (s_pout = tile-relative
// output offset of each piece, s_psrc = ABSOLUTE device address of its first byte; a sentinel
// s_pout[total_p] = tile output length) is in LDS; a block -> piece table is built, then lane i
// assembles aligned 16-byte output blocks i, i+blockDim, ...  Returns false (nothing written) when
// the piece table did not fit (the caller's slow path runs instead).
// PIPE: the pipelined interior loop (k_redact: 518 -> 506 us at config 2; the window re-scan's
// k_win_redact, whose tiles gather ring entries, measured slower with it: 84 -> 89 us, so it keeps the
// one-block loop)
template <bool PIPE>
__device__ __forceinline__ void tile_assemble(const uint32_t* s_pout, const uint64_t* s_psrc, uint32_t total_p,
                                              uint16_t* s_bp, uint32_t* s_wsum, uint8_t* __restrict__ out,
                                              int64_t out_lo, int64_t out_hi) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t omis = (int64_t)((uintptr_t)out & 15);
    const int64_t q_lo = (out_lo + omis) >> 4;
    const int64_t q_hi = out_hi > out_lo ? (out_hi - 1 + omis) >> 4 : q_lo - 1;
    const int64_t nblk = q_hi - q_lo + 1;
    const bool table = nblk > 0 && nblk <= BLK_MAX;
    if (table) {
        // block b's first valid byte is rf(b) = max(0, 16b - e0); piece(b) = max{p : pout[p] <= rf(b)}
        const uint32_t e0 = (uint32_t)((out_lo + omis) - 16 * q_lo);
        constexpr int PER = BLK_MAX / REDACT_BLOCK;
        for (int i = tid; i < BLK_MAX; i += REDACT_BLOCK) s_bp[i] = 0;
        __syncthreads();
        for (uint32_t p = tid; p < total_p; p += REDACT_BLOCK) {
            const uint32_t k = s_pout[p] == 0 ? 0u : (s_pout[p] + e0 + 15) >> 4;
            const uint32_t kn = p + 1 == total_p ? 0xffffffffu : (s_pout[p + 1] == 0 ? 0u : (s_pout[p + 1] + e0 + 15) >> 4);
            if (kn != k && k < (uint32_t)nblk) s_bp[k] = (uint16_t)p;      // last piece with this key
        }
        __syncthreads();
        // prefix max over the block table: PER entries per lane, then across lanes
        uint32_t m = 0;
        for (int j = 0; j < PER; ++j) m = max(m, (uint32_t)s_bp[tid * PER + j]);
        uint32_t incl_m = m;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl_m, d);
            if (lane >= d) incl_m = max(incl_m, o);
        }
        if (lane == 63) s_wsum[wid] = incl_m;
        __syncthreads();
        uint32_t run = 0;
        for (int w = 0; w < wid; ++w) run = max(run, s_wsum[w]);
        const uint32_t excl_m = __shfl_up(incl_m, 1);
        run = max(run, lane ? excl_m : 0u);
        for (int j = 0; j < PER; ++j) {
            run = max(run, (uint32_t)s_bp[tid * PER + j]);
            s_bp[tid * PER + j] = (uint16_t)run;
        }
        __syncthreads();
    }
    if (total_p == 0) return;
#if REDACT_ABLATE == 2
    return;                          // (measurement: tables only)
#endif
    uint4* __restrict__ op = reinterpret_cast<uint4*>(out - omis);
    const int64_t span = out_hi - out_lo;
    // a block's first piece is loaded before the loop over its further pieces (those are rare); two
    // or four blocks per thread in flight measured slower (more VGPRs, no fewer stalls)
    struct Blk {
        int64_t r0;
        int b_lo, b_hi, lo, hi;
        uint32_t pi, qs, qe;
        uint64_t qsrc;
        uint4 w;
    };
    auto begin = [&](Blk& k, int64_t q) {
        k.r0 = q * 16 - omis - out_lo;                   // tile-relative output offset of byte 0
        k.b_lo = k.r0 < 0 ? (int)-k.r0 : 0;              // valid bytes [b_lo, b_hi) of the block
        k.b_hi = k.r0 + 16 > span ? (int)(span - k.r0) : 16;
        if (table) {
            k.pi = s_bp[q - q_lo];
        } else {
            const uint32_t rs = (uint32_t)(k.r0 + k.b_lo);
            uint32_t lo_i = 0, hi_i = total_p - 1;       // last piece with s_pout <= rs
            while (lo_i < hi_i) {
                const uint32_t mid = (lo_i + hi_i + 1) >> 1;
                if (s_pout[mid] <= rs) lo_i = mid;
                else hi_i = mid - 1;
            }
            k.pi = lo_i;
        }
        k.qs = s_pout[k.pi];
        k.qe = s_pout[k.pi + 1];
        k.qsrc = s_psrc[k.pi];
        k.lo = max(k.b_lo, (int)((int64_t)k.qs - k.r0));
        k.hi = min(k.b_hi, (int)((int64_t)k.qe - k.r0));
        k.w = make_uint4(0, 0, 0, 0);
        if (k.hi > k.lo) k.w = load16(reinterpret_cast<const uint8_t*>(k.qsrc) + (k.r0 - (int64_t)k.qs), k.lo, k.hi);
    };
    auto merge = [](uint4& v, const uint4& w, int lo, int hi) {
        v.x |= w.x & (bytemask(hi) & ~bytemask(lo));
        v.y |= w.y & (bytemask(hi - 4) & ~bytemask(lo - 4));
        v.z |= w.z & (bytemask(hi - 8) & ~bytemask(lo - 8));
        v.w |= w.w & (bytemask(hi - 12) & ~bytemask(lo - 12));
    };
    auto finish = [&](Blk& k, int64_t q) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k.hi > k.lo) {
            if (k.lo == 0 && k.hi == 16) v = k.w;
            else merge(v, k.w, k.lo, k.hi);
        }
        while ((int64_t)k.qe < k.r0 + k.b_hi) {          // pieces overlapping [r0 + b_lo, r0 + b_hi)
            ++k.pi;
            k.qs = k.qe;
            k.qe = s_pout[k.pi + 1];
            k.qsrc = s_psrc[k.pi];
            const int lo = max(k.b_lo, (int)((int64_t)k.qs - k.r0));
            const int hi = min(k.b_hi, (int)((int64_t)k.qe - k.r0));
            if (hi > lo) merge(v, load16(reinterpret_cast<const uint8_t*>(k.qsrc) + (k.r0 - (int64_t)k.qs), lo, hi), lo, hi);
        }
        if (k.b_lo == 0 && k.b_hi == 16) {
            u32x4_t nv = {v.x, v.y, v.z, v.w};          // (streaming stores: -15 us per config-2 step)
            __builtin_nontemporal_store(nv, reinterpret_cast<u32x4_t*>(op + q));
        } else {
            uint8_t* ob = out - omis + q * 16;
            const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (j >= k.b_lo && j < k.b_hi) ob[j] = (uint8_t)(vw[j >> 2] >> (8 * (j & 3)));
        }
    };
#if REDACT_PIPE
    if (PIPE && table) {
        // Interior blocks (all 16 bytes in [out_lo, out_hi)) in a software pipeline: block q + 256's
        // piece lookup and its two source loads are issued before block q is merged and stored.  Every
        // load and store is unconditional (a chunk holding no byte of the piece is replaced by the
        // chunk that does, so no address leaves the source buffer), so the compiler's vmcnt waits are
        // counted and the next block's loads stay in flight -- a conditional load makes every wait a
        // vmcnt(0) (why two-blocks-per-iteration forms measured slower in rounds 3-4).  A block whose
        // bytes come from several pieces (~3% of them: the blocks around a token) is stored from its
        // first piece here and rebuilt by the general path after the loop (same thread, later store).
        const int64_t qa = q_lo + (((out_lo + omis) & 15) ? 1 : 0);
        const int64_t qb = q_hi - (((out_hi + omis) & 15) ? 1 : 0);
        struct Fast {
            uint4 x, y;
            uint32_t sh;
            bool one;
        };
        static_assert(BLK_MAX / REDACT_BLOCK <= 32, "fix mask: one bit per interior block of a thread");
        auto fetch = [&](Fast& f, int64_t q) {
            const uint32_t pi = s_bp[q - q_lo];
            const int64_t r0 = q * 16 - omis - out_lo;
            const uint32_t qs = s_pout[pi], qe = s_pout[pi + 1];
            const uintptr_t a = (uintptr_t)s_psrc[pi] + (uintptr_t)(r0 - (int64_t)qs);
            const uintptr_t a0 = a & ~(uintptr_t)15;
            f.sh = (uint32_t)(a & 15);
            f.one = (int64_t)qe >= r0 + 16;
            const bool two = f.sh + (f.one ? 16u : (uint32_t)((int64_t)qe - r0)) > 16u;
#if REDACT_ABLATE == 3
            f.x = make_uint4((uint32_t)a0, 0, 0, 0);      // (measurement: no source loads)
            f.y = f.x;
            (void)two;
#else
            f.x = gload16(a0);
            f.y = gload16(two ? a0 + 16 : a0);
#endif
        };
        uint32_t fix = 0;                 // bit i: this thread's i-th interior block needs the general path
        const int64_t q0 = qa + tid;
        if (q0 <= qb) {
            // ping-pong buffers (no register copy: a copy would wait for the loads it copies); past
            // the thread's last block a buffer re-reads and re-stores that block (the same bytes)
            const int64_t ql = q0 + ((qb - q0) / REDACT_BLOCK) * REDACT_BLOCK;
            auto put = [&](const Fast& f, int64_t q) {
                const uint4 v = window16(f.x, f.y, f.sh);
                u32x4_t nv = {v.x, v.y, v.z, v.w};
#if REDACT_NT
                __builtin_nontemporal_store(nv, reinterpret_cast<u32x4_t*>(op + q));
#else
                *reinterpret_cast<u32x4_t*>(op + q) = nv;
#endif
                if (!f.one) fix |= 1u << (uint32_t)((q - q0) / REDACT_BLOCK);
            };
            Fast f0, f1;
            fetch(f0, q0);
            for (int64_t q = q0; q <= ql; q += 2 * REDACT_BLOCK) {
                const int64_t q1 = min<int64_t>(q + REDACT_BLOCK, ql), q2 = min<int64_t>(q + 2 * REDACT_BLOCK, ql);
                fetch(f1, q1);
                put(f0, q);
                fetch(f0, q2);
                put(f1, q1);
            }
        }
        // the edge blocks and the multi-piece ones
        if (tid == 0 && qa > q_lo) {
            Blk k;
            begin(k, q_lo);
            finish(k, q_lo);
        }
        if (tid == REDACT_BLOCK - 1 && qb < q_hi && q_hi >= qa) {
            Blk k;
            begin(k, q_hi);
            finish(k, q_hi);
        }
        for (; fix; fix &= fix - 1) {
            const int64_t qf = qa + tid + (int64_t)__builtin_ctz(fix) * REDACT_BLOCK;
            Blk k;
            begin(k, qf);
            finish(k, qf);
        }
        return;
    }
#endif
    for (int64_t q = q_lo + tid; q <= q_hi; q += REDACT_BLOCK) {
        Blk k;
        begin(k, q);
        finish(k, q);
    }
}

// Per lane: its findings -> the API span list (pii_span at lane_sp[c] + k, batch order = (utterance,
// start) order) and the RSpan list; per-workgroup per-type histogram partials.  A finding's output
// position = its utterance's output offset + its start + the deltas of the utterance's earlier
// findings (for a cut row, starting from lane_rowbase: the row's findings in earlier lanes).
// Wave-cooperative (as k_pairs_flat): the 64 lanes' findings are one flattened list, 64 at a time --
// finding f belongs to the first lane whose inclusive count exceeds f, the running delta is a
// segmented scan over (lane, utterance) runs plus each lane's carry from the previous 64, and one
// store instruction writes 64 neighbouring records (the per-lane walk wrote record k of 64 lanes).
__global__ __launch_bounds__(256) void k_spans(const RulesDev R, const Geo g, const pii_span* __restrict__ fd,
                                               const uint32_t* __restrict__ lane_nf,
                                               const uint64_t* __restrict__ lane_sp,
                                               const int32_t* __restrict__ lane_rowbase,
                                               const uint64_t* __restrict__ out_offs, const uint32_t* __restrict__ err,
                                               pii_span* __restrict__ spans, RSpan* __restrict__ rsp,
                                               uint32_t* __restrict__ hist_part, uint32_t hist_types) {
    __shared__ uint32_t sh_hist[1024];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool run = *err == 0;
    for (uint32_t i = threadIdx.x; i < hist_types; i += blockDim.x) sh_hist[i] = 0;
    __syncthreads();
    const uint32_t nf = run && c < g.n_chunks ? lane_nf[c] : 0u;
    uint64_t fb = 0, sp0 = 0;            // the lane's findings arena, its first span index
    uint32_t cu0 = 0xffffffffu;          // a lane cut at lo: the cut row (its running delta starts at rb)
    int32_t rb = 0;
    if (nf) {
        const Lane L = g_lane(g, c);
        fb = fd_base(L, c, R.min_len);
        sp0 = lane_sp[c];
        if (L.clo) {
            cu0 = L.u0;
            rb = lane_rowbase[c];
        }
    }
    uint32_t incl = nf;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    const uint32_t total = __shfl(incl, 63), excl = incl - nf;
    uint32_t carry_u = 0xffffffffu;      // lane: utterance of its last finding handled, running delta after it
    int64_t carry_run = 0;
    for (uint32_t f0 = 0; f0 < total; f0 += 64) {
        const uint32_t f = f0 + lane;
        const bool act = f < total;
        int ow = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
            const uint32_t v = __shfl(incl, ow + step - 1);
            if (v <= f) ow += step;
        }
        const uint32_t o_ex = __shfl(excl, ow), o_cu0 = __shfl(cu0, ow), o_cu = __shfl(carry_u, ow);
        const int32_t o_rb = __shfl(rb, ow);
        const int64_t o_crun = __shfl(carry_run, ow);
        const uint64_t o_fb = __shfl(fb, ow), o_sp = __shfl(sp0, ow);
        const uint32_t k = f - o_ex;
        pii_span F{};
        int64_t d = 0;
        uint32_t t = 0;
        if (act) {
            F = fd[o_fb + k];
            t = F.info_type;
            d = (int64_t)(R.tok_off[t + 1] - R.tok_off[t]) - (int64_t)(F.end - F.start);
        }
        const uint32_t uk = act ? F.utt : 0xffffffffu;
        // running delta before this finding: its (lane, utterance) run's base + the run's earlier deltas
        int64_t sc = d;
#pragma unroll
        for (int dl = 1; dl < 64; dl <<= 1) {
            const int64_t o = __shfl_up(sc, dl);
            const int oo = __shfl_up(ow, dl);
            const uint32_t ou = __shfl_up(uk, dl);
            if (lane >= dl && oo == ow && ou == uk) sc += o;
        }
        const int64_t base = uk == o_cu ? o_crun : (uk == o_cu0 ? (int64_t)o_rb : 0);
        if (act) {
            spans[o_sp + k] = F;
            const int64_t ubase_in = g_off(g, F.utt), ubase_out = (int64_t)out_offs[F.utt];
            RSpan rs;
            rs.in_lo = (uint32_t)(ubase_in + F.start);
            rs.in_hi = (uint32_t)(ubase_in + F.end);
            rs.out = (uint64_t)(ubase_out + F.start + base + (sc - d)) | ((uint64_t)t << 48);
            rsp[o_sp + k] = rs;
            if (t < hist_types) atomicAdd(&sh_hist[t], 1u);
        }
        // each lane carries the utterance and running delta of its last finding in this chunk
        const bool here = nf && incl > f0 && excl < f0 + 64;
        const int last = here ? (int)(min(incl, f0 + 64) - 1 - f0) : 0;
        const uint32_t lu = __shfl(uk, last);
        const int64_t lrun = __shfl(base + sc, last);
        if (here) {
            carry_u = lu;
            carry_run = lrun;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < hist_types; i += blockDim.x)
        hist_part[(size_t)i * gridDim.x + blockIdx.x] = sh_hist[i];
}

__device__ __forceinline__ uint64_t rs_out(const RSpan& r) { return r.out & 0xffffffffffffull; }
__device__ __forceinline__ uint32_t rs_type(const RSpan& r) { return (uint32_t)(r.out >> 48); }

// first span whose token ends after the tile's first output byte (binary search, one thread per tile)
__global__ __launch_bounds__(256) void k_tile_first(const RulesDev R, const RSpan* __restrict__ rsp,
                                                    const uint64_t* __restrict__ n_spans_p,
                                                    const uint64_t* __restrict__ out_total_p, uint32_t omis,
                                                    uint32_t max_tiles, const uint32_t* __restrict__ err,
                                                    uint32_t* __restrict__ tile_first) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= max_tiles || *err) return;
    const int64_t lo = ((int64_t)k << RTILE_SHIFT) - omis;
    if (lo >= (int64_t)*out_total_p) return;
    uint64_t a = 0, b = *n_spans_p;          // first i in [a, b) with token end > lo
    while (a < b) {
        const uint64_t m = (a + b) >> 1;
        const RSpan r = rsp[m];
        const uint32_t t = rs_type(r);
        if ((int64_t)(rs_out(r) + (R.tok_off[t + 1] - R.tok_off[t])) > lo) b = m;
        else a = m + 1;
    }
    tile_first[k] = (uint32_t)a;
}

__global__ __launch_bounds__(REDACT_BLOCK) void k_redact(const RulesDev R, const uint8_t* __restrict__ text,
                                                         const uint64_t* __restrict__ offs,
                                                         const RSpan* __restrict__ rsp,
                                                         const uint64_t* __restrict__ n_spans_p,
                                                         const uint64_t* __restrict__ out_total_p, uint64_t in_total,
                                                         const uint32_t* __restrict__ tile_first,
                                                         const uint32_t* __restrict__ err, uint8_t* __restrict__ out) {
    __shared__ uint32_t s_pout[PIECE_MAX + 1];     // piece output offset (pass relative)
    __shared__ uint64_t s_psrc[PIECE_MAX + 1];     // piece source address (text or token table)
    __shared__ uint32_t s_wsum[REDACT_BLOCK / 64];
    __shared__ uint16_t s_bp[BLK_MAX];             // output block -> piece holding its first byte
    if (*err != 0) return;
    const int64_t out_total = (int64_t)*out_total_p;
    const uint64_t n_spans = *n_spans_p;
    const int64_t omis = (int64_t)((uintptr_t)out & 15);
    const int64_t t_lo = max<int64_t>(((int64_t)blockIdx.x << RTILE_SHIFT) - omis, 0);
    const int64_t t_hi = min<int64_t>(((int64_t)(blockIdx.x + 1) << RTILE_SHIFT) - omis, out_total);
    if (t_lo >= t_hi) return;
    const uint8_t* tb = text + offs[0];
    const int k = threadIdx.x;
    uint64_t i = tile_first[blockIdx.x];          // first span whose token ends after t_lo
    int64_t lo = t_lo;
    while (lo < t_hi) {
        // one pass: spans i .. i + n - 1 (their tokens start before the tile end; n <= SPAN_PASS);
        // piece 2k = the copy run before span i + k, 2k + 1 = its token, 2n = the run after the last
        const uint64_t j = i + (uint64_t)k;
        RSpan r{0, 0, 0};
        bool mine = false;
        if (k < SPAN_PASS && j < n_spans) {
            r = rsp[j];
            mine = (int64_t)rs_out(r) < t_hi;
        }
        const uint32_t n = (uint32_t)__syncthreads_count(mine);
        int64_t hi = t_hi;                            // a full pass ends where the next token starts
        if (n == (uint32_t)SPAN_PASS && i + n < n_spans) hi = min<int64_t>(hi, (int64_t)rs_out(rsp[i + n]));
        if (mine) {
            const uint32_t ty = rs_type(r);
            const int64_t so = (int64_t)rs_out(r);
            const int64_t tl = (int64_t)(R.tok_off[ty + 1] - R.tok_off[ty]);
            if (k == 0) {                             // from lo, shifted like the run before span i
                s_pout[0] = 0;
                s_psrc[0] = (uint64_t)(uintptr_t)(tb + (lo - (so - (int64_t)r.in_lo)));
            } else {                                  // from the previous token's end
                const RSpan pr = rsp[j - 1];
                const uint32_t pt = rs_type(pr);
                const int64_t pe = (int64_t)rs_out(pr) + (int64_t)(R.tok_off[pt + 1] - R.tok_off[pt]);
                s_pout[2 * k] = (uint32_t)(pe - lo);
                s_psrc[2 * k] = (uint64_t)(uintptr_t)(tb + pr.in_hi);
            }
            const int64_t ts = max(so, lo);
            s_pout[2 * k + 1] = (uint32_t)(ts - lo);
            s_psrc[2 * k + 1] = (uint64_t)(uintptr_t)(R.tok_bytes + R.tok_off[ty] + (ts - so));
            if ((uint32_t)k + 1 == n) {
                const int64_t te = min(so + tl, hi);
                s_pout[2 * n] = (uint32_t)(te - lo);
                s_psrc[2 * n] = (uint64_t)(uintptr_t)(tb + r.in_hi);
                s_pout[2 * n + 1] = (uint32_t)(hi - lo);           // sentinel
            }
        }
        if (n == 0 && k == 0) {                       // no token in [lo, hi): one copy run
            const int64_t shift = i < n_spans ? (int64_t)rs_out(rsp[i]) - (int64_t)rsp[i].in_lo
                                              : out_total - (int64_t)in_total;
            s_pout[0] = 0;
            s_psrc[0] = (uint64_t)(uintptr_t)(tb + (lo - shift));
            s_pout[1] = (uint32_t)(hi - lo);
        }
        __syncthreads();
#if REDACT_ABLATE != 1
        tile_assemble<true>(s_pout, s_psrc, n == 0 ? 1u : 2 * n + 1, s_bp, s_wsum, out, lo, hi);
#endif
        __syncthreads();
        i += n;
        lo = hi;
    }
}

// per-info-type totals of the redact tiles' histograms (one atomic per type, no same-address storms)
__global__ __launch_bounds__(256) void k_hist_reduce(const uint32_t* __restrict__ hist_part, uint32_t n_tiles, int T,
                                                     const uint32_t* __restrict__ err,
                                                     unsigned long long* __restrict__ hist) {
    __shared__ unsigned long long s_sum[4];
    if (*err != 0) return;                   // k_redact did not run: the call is reported as failed
    const int t = blockIdx.x;
    unsigned long long v = 0;
    for (uint32_t b = blockIdx.y * blockDim.x + threadIdx.x; b < n_tiles; b += gridDim.y * blockDim.x)
        v += hist_part[(size_t)t * n_tiles + b];
    for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d);
    if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long tot = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
        if (tot) atomicAdd(&hist[t], tot);
    }
}

// ============================================================================ window re-scan (a12)
// README.md:131-134 / SURVEY A.9: after each utterance the aggregator re-redacts "\n".join(last N
// utterances) with the conversation's current expected_pii_type.  Incremental form used here:
// when no detector can consume '\n' or test a text edge (compiler `window_ok`), a match inside the
// window lies inside one utterance and equals that utterance's own match, so each utterance is
// scanned ONCE (its new bytes), and its finditer-resolved, validator-passing candidates are kept
// resident in HBM with a bit per hotword rule for the proximity windows clipped to the utterance.
// A window then only (1) re-evaluates hotword windows that reach across a "\n" into a neighbour
// utterance (the halo), (2) applies the window's context variant (likelihoods, min likelihood,
// exclusion, overlap) and (3) writes the redacted window.  Candidates of different utterances never
// overlap, so exclusion and overlap resolution stay per utterance.
constexpr int WN_MAX = 8;          // largest window (utterances)
constexpr int WIN_TILE = 64;       // windows per k_win_redact workgroup

constexpr int WHOT_BITS = 16;      // hotword rules whose proximity results are kept resident
#ifndef WIN_HALO_ABLATE
#define WIN_HALO_ABLATE 0           // measurement builds only: 1 = no hotword DFA runs, 2 = row prologue only
#endif
struct WCand {          // one resident candidate (16 B)
    uint32_t s, e;      // match [s, e), relative to its utterance
    uint16_t p;         // detector pattern (any rule set: config 5 has 544)
    uint8_t need;       // predecessors its longest before-window needs (0: it stays inside the utterance)
    uint8_t pad;
    uint16_t hot;       // bit h: hotword rule h hits, proximity windows clipped to the utterance
    uint16_t hotx;      // bit h: ... before-window over the (up to `need`) preceding utterances
};
static_assert(sizeof(WCand) == 16, "WCand is one 16-byte record in the ring arena");
struct WDesc {          // one resident utterance of a conversation's history ring (16 B)
    uint32_t off;       // arena offset (16-aligned): nc WCands, then the text bytes
    uint32_t len;
    uint32_t nc;
    uint32_t pad;
};
struct WNew {           // commit plan of a batch row that enters its conversation's ring
    uint32_t off;       // arena offset, ~0 = the row does not enter the ring
    uint32_t ri;        // descriptor index
    uint32_t cnt;       // (last row of a run) live entries after the commit
    uint32_t head;      // (last row of a run) next descriptor index after the commit
};
struct WinRing {        // per-conversation history in HBM (replaces the aggregator's Redis list)
    WDesc* desc;        // [slots * N]
    uint32_t* cnt;      // [slots] live entries (<= N)
    uint32_t* head;     // [slots] next descriptor index (newest = head - 1 mod N)
    uint8_t* arena;     // [slots * slot_bytes]
    uint32_t N, slot_bytes, n_slots, pad;
};
struct WinBatch {       // this call's rows and their freshly built candidate lists
    const uint8_t* text;
    const uint64_t* offs;
    const uint32_t* slot;
    const WCand* wc;
    const uint32_t* wc_first;
    const uint32_t* wc_n;
    uint32_t n_utt;
};
struct WEntry {
    const uint8_t* t;
    const WCand* c;
    uint32_t len, nc;
};

// The window of row u, oldest first: the r newest ring entries of u's conversation, then u's m
// same-conversation predecessors in the batch, then u.  Entries are produced on demand (win_at), so
// the kernels keep no per-thread entry arrays (which would live in scratch memory).
struct WinIt {
    uint32_t u, sl, m, r, head;
    int nw;
};

__device__ __forceinline__ WinIt win_begin(const WinRing& W, const WinBatch& B, uint32_t u) {
    WinIt it;
    it.u = u;
    it.sl = B.slot[u];
    uint32_t m = 0;
    while (m + 1 < W.N && u >= m + 1 && B.slot[u - m - 1] == it.sl) ++m;
    uint32_t r = 0, head = 0;
    if (m + 1 < W.N && it.sl < W.n_slots) {
        r = min(W.N - 1 - m, W.cnt[it.sl]);
        head = W.head[it.sl];
    }
    it.m = m;
    it.r = r;
    it.head = head;
    it.nw = (int)(r + m + 1);
    return it;
}

__device__ __forceinline__ WEntry win_at(const WinRing& W, const WinBatch& B, const WinIt& it, int j) {
    WEntry E;
    if ((uint32_t)j < it.r) {
        const WDesc D = W.desc[(size_t)it.sl * W.N + (it.head + W.N - it.r + (uint32_t)j) % W.N];
        const uint8_t* a = W.arena + (size_t)it.sl * W.slot_bytes + D.off;
        E.t = a + 16u * D.nc;
        E.c = reinterpret_cast<const WCand*>(a);
        E.len = D.len;
        E.nc = D.nc;
    } else {
        const uint32_t v = it.u - it.m + ((uint32_t)j - it.r);
        const uint64_t a = B.offs[v];
        E.t = B.text + a;
        E.nc = B.wc_n[v];
        E.c = B.wc + (E.nc ? B.wc_first[v] : 0u);
        E.len = (uint32_t)(B.offs[v + 1] - a);
    }
    return E;
}

// Unanchored HOT DFA over window positions [lo, hi) (entries joined by '\n'), window edges as text
// edges: the proximity test of a candidate whose window reaches into a neighbour utterance.
__device__ bool hot_run_win(const Pool& pool, const int32_t* d, const WinRing& W, const WinBatch& B,
                            const WinIt& it, uint32_t lo, uint32_t hi) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* cm = pool.cmap + d[2];
    const uint32_t nc = (uint32_t)d[3];
    uint32_t st = (uint32_t)d[4];
    uint32_t sl = 0;
    for (int j = 0; j < it.nw; ++j) {
        const WEntry Ej = win_at(W, B, it, j);
        const uint32_t sh = sl + Ej.len;
        if (sh >= lo) {
            if (sl >= hi) break;
            const int a = (int)(max(lo, sl) - sl), b = (int)(min(hi, sh) - sl);
            if (hot_span(tr, cm, nc, Ej.t, a, b, st)) return true;
            if (j + 1 < it.nw && sh < hi) {
                const uint32_t x = tr[st * nc + cm['\n']];
                if (x & 0x4000u) return true;
                st = x & DFA_STATE_MASK;
            }
        }
        sl = sh + 1;
    }
    return (tr[st * nc + nc - 1] & 0x4000u) != 0;
}

// hot_span over text[lo, hi) with every chunk of a short window (<= 64 bytes) loaded before the first
// step (hot_span loads the next 16 bytes only after stepping the current ones)
__device__ __forceinline__ bool hot_span_pre(const uint16_t* tr, const uint8_t* cm, uint32_t nc, const uint8_t* text,
                                             int lo, int hi, uint32_t& st) {
    if (hi - lo > 64) return hot_span(tr, cm, nc, text, lo, hi, st);
    uint4 w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int j = lo + 16 * c;
        w[c] = make_uint4(0, 0, 0, 0);
        if (j < hi) w[c] = load16(text + j, 0, hi - j < 16 ? hi - j : 16);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int j = lo + 16 * c;
        if (j >= hi) break;
        const int n = hi - j < 16 ? hi - j : 16;
        uint4 x = w[c];
#pragma unroll 1
        for (int g = 0; g < n; g += 4) {
            const uint32_t v = x.x;
            const uint32_t cl[4] = {cm[v & 0xffu], cm[(v >> 8) & 0xffu], cm[(v >> 16) & 0xffu], cm[v >> 24]};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (g + k < n) {
                    const uint32_t e = tr[st * nc + cl[k]];
                    if (e & 0x4000u) return true;
                    st = e & DFA_STATE_MASK;
                }
            }
            x = make_uint4(x.y, x.z, x.w, 0u);
        }
    }
    return false;
}

// per matched pair: validator + every hotword rule the pattern's type has in ANY context variant,
// proximity windows clipped to the utterance -> PairRes.lik = 0 valid / -1 invalid, phot = rule bits
template <bool GI>
__global__ __launch_bounds__(PAIR_BLOCK) void k_win_eval(const uint4* __restrict__ img, const LdsImage li,
                                                         const uint8_t* __restrict__ text0,
                                                         const uint64_t* __restrict__ offs,
                                                         const unsigned long long* __restrict__ pair_count,
                                                         uint64_t pair_cap, const uint32_t* __restrict__ matched,
                                                         const uint32_t* __restrict__ mcount, uint32_t nseg,
                                                         const EvLoc* __restrict__ evloc,
                                                         const int32_t* __restrict__ pend,
                                                         PairRes* __restrict__ pres, uint32_t* __restrict__ phot) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    const Pool pool{reinterpret_cast<const uint16_t*>(lb + li.off[EV_TRANS]), lb + li.off[EV_CMAP]};
    const int32_t* hdesc = reinterpret_cast<const int32_t*>(lb + li.off[EV_HDESC]);
    const int32_t* hrule = reinterpret_cast<const int32_t*>(lb + li.off[EV_HRULE]);
    const uint16_t* dtype = reinterpret_cast<const uint16_t*>(lb + li.off[EV_DTYPE]);
    const uint8_t* dval = lb + li.off[EV_DVAL];
    const uint32_t* thot = reinterpret_cast<const uint32_t*>(lb + li.off[EV_THOT]);
    const uint8_t* text = text0 + offs[0];
    __shared__ uint32_t s_mp[PAIR_WAVES + 1];
    const uint64_t seg = pair_segment(min((uint64_t)*pair_count, pair_cap), nseg * PAIR_WAVES);
    for (uint32_t g = blockIdx.x; g < nseg; g += gridDim.x) {
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int w = 0; w < PAIR_WAVES; ++w) {
                s_mp[w] = run;
                run += mcount[g * PAIR_WAVES + w];
            }
            s_mp[PAIR_WAVES] = run;
        }
        __syncthreads();
        const uint32_t m = s_mp[PAIR_WAVES];
        for (uint32_t k = threadIdx.x; k < m; k += blockDim.x) {
            int w = 0;
            while (w + 1 < PAIR_WAVES && s_mp[w + 1] <= k) ++w;
            const uint32_t i = matched[(uint64_t)(g * PAIR_WAVES + w) * seg + (k - s_mp[w])];
            const PairRes P = pres[i];
            const EvLoc Lc = evloc[P.ev];
            const uint8_t* t0 = text + Lc.ustart;
            const int L = (int)(Lc.uend - Lc.ustart);
            const int s = (int)(Lc.s - Lc.ustart), e = pend[i];
            int lik = -1;
            uint32_t hot = 0;
            if (validate(dval[P.p], t0 + s, e - s)) {
                lik = 0;
                uint32_t mask = thot[dtype[P.p]];
                while (mask) {
                    const int h = __builtin_ctz(mask);
                    mask &= mask - 1;
                    const int wb = hrule[4 * h], wa = hrule[4 * h + 1];
                    bool hit = false;
                    if (wb > 0) hit = hot_run(pool, hdesc + 8 * h, t0, s - wb > 0 ? s - wb : 0, s);
                    if (!hit && wa > 0) hit = hot_run(pool, hdesc + 8 * h, t0, e, e + wa < L ? e + wa : L);
                    if (hit) hot |= 1u << h;
                }
            }
            pres[i].lik = (int16_t)lik;
            phot[i] = hot;
        }
    }
}

// per scan lane: finditer skipping per pattern over the lane's matched pairs (variant independent),
// then the validator-passing survivors become the rows' resident candidates (wc, in pair-queue slots
// of the lane: a lane never has more candidates than pairs)
// leading pairs of lane c that belong to row r (a row cut at the lane's lo): the lane's pairs are in
// position order, so a binary search over their rows
__device__ __forceinline__ uint32_t lead_pairs(const PairRes* __restrict__ pres, const EvLoc* __restrict__ evloc,
                                               uint64_t base, uint32_t np, uint32_t r) {
    uint32_t lo = 0, hi = np;                      // first pair whose row is not r
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (evloc[pres[base + mid].ev].u == r) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_win_cands(const Geo g, const uint64_t* __restrict__ lane_pair,
                                                   const uint32_t* __restrict__ lane_np,
                                                   const EvLoc* __restrict__ evloc, const PairRes* __restrict__ pres,
                                                   const int32_t* __restrict__ pend, const uint32_t* __restrict__ phot,
                                                   uint64_t pair_cap, uint2* __restrict__ spill, WCand* __restrict__ wc,
                                                   uint32_t* __restrict__ wc_first, uint32_t* __restrict__ wc_n,
                                                   const uint32_t* __restrict__ err) {
    if (*err & ERR_ABORT) return;
    const uint32_t n_chunks = g.n_chunks;
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    const Lane L = g_lane(g, c);
    const uint32_t np0 = lane_np[c];
    if (lane_pair[c] + np0 > pair_cap) return;
    // A row cut into several lanes (rows longer than long_min) is walked whole by the thread of the
    // lane holding its start: it continues into the next lanes' leading pairs, which their own
    // threads skip.  Its candidates and spill list run on past the lane's slots into the next lanes'
    // (never further than the pairs it has walked), so a lane's own rows start behind the skipped ones.
    const uint32_t i0 = L.clo ? lead_pairs(pres, evloc, lane_pair[c], np0, L.u0) : 0u;
    const uint64_t base = lane_pair[c] + i0;       // this thread's wc / spill slots
    const uint32_t np = np0 - i0;
    uint32_t u = 0xffffffffu, k = 0, uf = 0;
    int lp[LIVE], le[LIVE];
    // more than LIVE patterns live in one row: their (pattern, end) list in the lane's pair-queue slots
    // of `spill` (k_select's buffer, unused on the window path), as in select_run
    uint2* __restrict__ sp = spill + base;
    uint32_t n_spill = 0;
    bool spilled = false;
#pragma unroll
    for (int q = 0; q < LIVE; ++q) {
        lp[q] = -1;
        le[q] = -1;
    }
    auto cand = [&](uint64_t pi, int e) {            // pi: pair index
        const PairRes P = pres[pi];
        const EvLoc Lc = evloc[P.ev];
        const int s = (int)(Lc.s - Lc.ustart);
        if (Lc.u != u) {
            if (u != 0xffffffffu && k > uf) {
                wc_first[u] = (uint32_t)(base + uf);
                wc_n[u] = k - uf;
            }
            u = Lc.u;
            uf = k;
#pragma unroll
            for (int q = 0; q < LIVE; ++q) {
                lp[q] = -1;
                le[q] = -1;
            }
            spilled = false;
        }
        const int p = P.p;
        int prev_end = -1;
        if (spilled) {
            for (uint32_t q = 0; q < n_spill; ++q)
                if ((int)sp[q].x == p) prev_end = (int)sp[q].y;
        } else {
#pragma unroll
            for (int q = 0; q < LIVE; ++q)
                if (lp[q] == p) prev_end = le[q];
        }
        if (s < prev_end) return;                    // inside p's previous match (finditer)
        if (spilled) {
            uint32_t q = 0;
            while (q < n_spill && (int)sp[q].x != p) ++q;
            sp[q] = make_uint2((uint32_t)p, (uint32_t)e);
            if (q == n_spill) ++n_spill;
        } else {
            int slot = -1;
#pragma unroll
            for (int q = 0; q < LIVE; ++q)
                if (lp[q] == p) slot = q;
            if (slot < 0) {
#pragma unroll
                for (int q = 0; q < LIVE; ++q)
                    if (slot < 0 && le[q] <= s) slot = q;
            }
            if (slot >= 0) {
#pragma unroll
                for (int q = 0; q < LIVE; ++q)
                    if (q == slot) {
                        lp[q] = p;
                        le[q] = e;
                    }
            } else {
                n_spill = 0;
#pragma unroll
                for (int q = 0; q < LIVE; ++q)
                    if (lp[q] >= 0) sp[n_spill++] = make_uint2((uint32_t)lp[q], (uint32_t)le[q]);
                sp[n_spill++] = make_uint2((uint32_t)p, (uint32_t)e);
                spilled = true;
            }
        }
        if (P.lik < 0) return;                       // validator failed
        WCand C;
        C.s = (uint32_t)s;
        C.e = (uint32_t)e;
        C.p = (uint16_t)p;
        C.need = 0;
        C.pad = 0;
        C.hot = (uint16_t)phot[pi];
        C.hotx = C.hot;
        wc[base + k++] = C;
    };
    // the matched pairs of the pend[] run [pb, pb + n) in prefetched 16-entry groups (as in k_select)
    auto walk = [&](uint64_t pb, uint32_t n) {
        if (n == 0) return;
        const uint32_t off0 = (uint32_t)(pb & 3u);
        const int4* pa = reinterpret_cast<const int4*>(pend + (pb - off0));
        const uint32_t ng = (off0 + n + 15u) >> 4;
        int4 q0 = pa[0], q1 = pa[1], q2 = pa[2], q3 = pa[3];
        for (uint32_t gi = 0; gi < ng; ++gi) {
            const int4 c0 = q0, c1 = q1, c2 = q2, c3 = q3;
            if (gi + 1 < ng) {
                const int4* pn = pa + 4 * (gi + 1);
                q0 = pn[0];
                q1 = pn[1];
                q2 = pn[2];
                q3 = pn[3];
            }
            const uint32_t g0 = 16u * gi;
            uint32_t m = matched_mask16(c0, c1, c2, c3, g0, off0, n);
            while (m) {
                const uint32_t j = (uint32_t)__builtin_ctz(m);
                m &= m - 1u;
                const uint64_t pi = pb + (g0 + j - off0);
                cand(pi, pend[pi]);
            }
        }
    };
    walk(base, np);
    // the lane's last row continues into the next lanes: their leading pairs
    if (L.chi) {
        const uint32_t r = L.u1 - 1;
        for (uint32_t c2 = c + 1; c2 < n_chunks; ++c2) {
            const uint32_t n2 = lane_np[c2];
            const uint64_t b2 = lane_pair[c2];
            if (b2 + n2 > pair_cap) break;
            walk(b2, lead_pairs(pres, evloc, b2, n2, r));
            const Lane L2 = g_lane(g, c2);
            if (!(L2.chi && L2.u1 - 1 == r)) break;
        }
    }
    if (u != 0xffffffffu && k > uf) {
        wc_first[u] = (uint32_t)(base + uf);
        wc_n[u] = k - uf;
    }
}

// per NEW row: the before-windows of its candidates that reach across the "\n" into the preceding
// utterances are evaluated ONCE, here, over the predecessors the row's own window holds (those are
// the only ones any later window can hold before it): hotx + need.  A later window in which the
// utterance has j >= need predecessors reuses hotx; j == 0 (window start) reuses hot.
// Two phases per workgroup of HALO_ROWS rows.  Phase 1, a thread per row: the row's window entries
// (text, length, counted back from the row) into LDS, need written, and one ITEM per (candidate,
// hotword rule) whose before-window must be re-run, appended to the workgroup's LDS list.  Phase 2:
// the items spread over all threads, one DFA run each, hits ORed into hotx.  (One thread running all
// of its row's items: a wavefront took as long as its busiest row's candidates x rules x window
// steps, 83 us per config-3 step at 0.8 waves / SIMD; two threads per row: 49 us.)
constexpr int HALO_ROWS = 256, HALO_ITEMS = 1024;
constexpr uint32_t HALO_LDS = HALO_ROWS * WN_MAX * 12 + HALO_ROWS * 12 + HALO_ITEMS * 8 + 16;

// hot_run_win over a row's LDS window table (rt / rl: the entries counted back from the row, 0 = the
// row itself, j = the oldest)
__device__ __forceinline__ bool hot_run_back(const Pool& pool, const int32_t* d, const uint64_t* rt, const uint32_t* rl,
                                             int j, uint32_t lo, uint32_t hi) {
    const uint16_t* tr = pool.trans + d[0];
    const uint8_t* cm = pool.cmap + d[2];
    const uint32_t nc = (uint32_t)d[3];
    uint32_t st = (uint32_t)d[4];
    uint32_t sl = 0;
    for (int i = j; i >= 0; --i) {
        const uint32_t sh = sl + rl[i];
        if (sh >= lo) {
            if (sl >= hi) break;
            const int a = (int)(max(lo, sl) - sl), b = (int)(min(hi, sh) - sl);
            if (hot_span_pre(tr, cm, nc, reinterpret_cast<const uint8_t*>(rt[i]), a, b, st)) return true;
            if (i > 0 && sh < hi) {
                const uint32_t x = tr[st * nc + cm['\n']];
                if (x & 0x4000u) return true;
                st = x & DFA_STATE_MASK;
            }
        }
        sl = sh + 1;
    }
    return (tr[st * nc + nc - 1] & 0x4000u) != 0;
}

template <bool GI>
__global__ __launch_bounds__(HALO_ROWS) void k_win_halo(const uint4* __restrict__ img, const LdsImage li, const WinRing W,
                                                        const WinBatch B, WCand* __restrict__ wc, uint32_t item_cap,
                                                        const uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    if (*err & (ERR_ABORT | ERR_SLOT)) return;
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    const Pool pool{reinterpret_cast<const uint16_t*>(lb + li.off[EV_TRANS]), lb + li.off[EV_CMAP]};
    const int32_t* hdesc = reinterpret_cast<const int32_t*>(lb + li.off[EV_HDESC]);
    const int32_t* hrule = reinterpret_cast<const int32_t*>(lb + li.off[EV_HRULE]);
    const uint16_t* dtype = reinterpret_cast<const uint16_t*>(lb + li.off[EV_DTYPE]);
    const uint32_t* thot = reinterpret_cast<const uint32_t*>(lb + li.off[EV_THOT]);
    // item_cap <= HALO_ITEMS (smaller only in tests: PII_HALO_ITEMS, the list-full path)
    // the tables after the image (dynamic LDS: image bytes rounded up to 16, then HALO_LDS)
    uint8_t* hb0 = reinterpret_cast<uint8_t*>(lds4) + (GI ? 0u : (li.total + 15u) & ~15u);
    uint64_t* s_rt = reinterpret_cast<uint64_t*>(hb0);                            // [row][WN_MAX]
    uint32_t* s_rl = reinterpret_cast<uint32_t*>(s_rt + HALO_ROWS * WN_MAX);       // [row][WN_MAX]
    uint64_t* s_cl = reinterpret_cast<uint64_t*>(s_rl + HALO_ROWS * WN_MAX);       // [row]: its candidates
    uint32_t* s_j = reinterpret_cast<uint32_t*>(s_cl + HALO_ROWS);                 // [row]: predecessors
    uint2* s_item = reinterpret_cast<uint2*>(s_j + HALO_ROWS);                     // (ps, row << 24 | k << 4 | rule)
    uint32_t* s_n = reinterpret_cast<uint32_t*>(s_item + HALO_ITEMS);
    const int tid = threadIdx.x;
    if (tid == 0) *s_n = 0;
    __syncthreads();
    const uint32_t u = blockIdx.x * HALO_ROWS + tid;
    const uint32_t nc = u < B.n_utt ? B.wc_n[u] : 0u;
    WinIt it;
    it.nw = 1;
    if (nc) it = win_begin(W, B, u);
    const int j = it.nw - 1;                       // predecessors available
    if (nc && j > 0) {
        WCand* cl = wc + B.wc_first[u];
        uint64_t* rt = s_rt + tid * WN_MAX;
        uint32_t* rl = s_rl + tid * WN_MAX;
        uint32_t oj = 0;                            // window offset of row u
        for (int i = 0; i <= j; ++i) {
            const WEntry E = win_at(W, B, it, j - i);
            rt[i] = (uint64_t)(uintptr_t)E.t;
            rl[i] = E.len;
            if (i >= 1) oj += E.len + 1;
        }
        s_cl[tid] = (uint64_t)(uintptr_t)cl;
        s_j[tid] = (uint32_t)j;
        for (uint32_t k = 0; k < nc; ++k) {
            const WCand C = cl[k];
            const uint32_t mask = thot[dtype[C.p]] & ((1u << WHOT_BITS) - 1);
            int wbmax = 0;
            for (uint32_t m = mask; m; m &= m - 1) wbmax = max(wbmax, hrule[4 * __builtin_ctz(m)]);
            if ((int)C.s >= wbmax) continue;
            // predecessors the longest before-window reaches (all available ones if it reaches past them)
            int need = 0;
            uint32_t cover = C.s;
            while (need < j && cover < (uint32_t)wbmax) {
                ++need;
                cover += rl[need] + 1;
            }
            cl[k].need = (uint8_t)need;
            const uint32_t ps = oj + C.s;
            uint32_t hx = 0;
            for (uint32_t m = mask & ~(uint32_t)C.hot; m; m &= m - 1) {
                const uint32_t hb = (uint32_t)__builtin_ctz(m);
                const int wb = hrule[4 * hb];
                if (wb <= 0 || (int)C.s >= wb) continue;
                const uint32_t q = atomicAdd(s_n, 1u);
                if (q < item_cap && k < (1u << 20)) {
                    s_item[q] = make_uint2(ps, (uint32_t)tid << 24 | k << 4 | hb);
                } else if (hot_run_back(pool, hdesc + 8 * hb, rt, rl, j, ps > (uint32_t)wb ? ps - wb : 0u, ps)) {
                    hx |= 1u << hb;                 // (list full: run here)
                }
            }
            if (hx) atomicOr(reinterpret_cast<uint32_t*>(cl + k) + 3, hx << 16);   // hotx (dword 3: hot | hotx << 16)
        }
    }
    __syncthreads();
    const uint32_t n = min(*s_n, item_cap);
    for (uint32_t q = tid; q < n; q += HALO_ROWS) {
        const uint2 I = s_item[q];
        const uint32_t r = I.y >> 24, k = (I.y >> 4) & 0xfffffu, hb = I.y & 15u;
        const uint32_t ps = I.x, wb = (uint32_t)hrule[4 * hb];
        if (hot_run_back(pool, hdesc + 8 * hb, s_rt + r * WN_MAX, s_rl + r * WN_MAX, (int)s_j[r], ps > wb ? ps - wb : 0u, ps)) {
            WCand* C = reinterpret_cast<WCand*>((uintptr_t)s_cl[r]) + k;
            atomicOr(reinterpret_cast<uint32_t*>(C) + 3, 1u << (16 + hb));
        }
    }
}

// per row: upper bound of its window's findings (= candidates in the window) for the findings arena;
// clears the row's ring-commit plan
__global__ __launch_bounds__(256) void k_win_plan(const WinRing W, const WinBatch B, uint32_t* __restrict__ bound,
                                                  WNew* __restrict__ wnew, const uint32_t* __restrict__ err) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= B.n_utt) return;
    WNew z;
    z.off = 0xffffffffu;
    z.ri = z.cnt = z.head = 0;
    wnew[u] = z;
    if (*err & (ERR_ABORT | ERR_SLOT)) {
        bound[u] = 0;
        return;
    }
    const WinIt it = win_begin(W, B, u);
    uint32_t b = 0;
    for (int j = 0; j < it.nw; ++j) b += win_at(W, B, it, j).nc;
    bound[u] = b;
}

// per window: the window's context variant -> hotword likelihoods (resident bits, or a re-run over
// the halo when a proximity window crosses a '\n'), min likelihood, exclusion, overlap; findings in
// window coordinates, output length
template <bool GI>
__global__ __launch_bounds__(256) void k_win_select(const RulesDev R, const uint4* __restrict__ img, const LdsImage li,
                                                    const WinRing W, const WinBatch B,
                                                    const int16_t* __restrict__ win_ctx,
                                                    const uint64_t* __restrict__ fbase, uint64_t fcap,
                                                    pii_span* __restrict__ wfd, uint32_t* __restrict__ n_wfind,
                                                    uint32_t* __restrict__ wout_len, uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds4[];
    if (*err & (ERR_ABORT | ERR_SLOT)) return;
    const uint8_t* lb = load_image<GI>(img, li.total, lds4);
    const Pool pool{reinterpret_cast<const uint16_t*>(lb + li.off[WS_TRANS]), lb + li.off[WS_CMAP]};
    const int32_t* hdesc = reinterpret_cast<const int32_t*>(lb + li.off[WS_HDESC]);
    const int32_t* hrule = reinterpret_cast<const int32_t*>(lb + li.off[WS_HRULE]);
    const uint16_t* dtype = reinterpret_cast<const uint16_t*>(lb + li.off[WS_DTYPE]);
    const uint8_t* dlik = lb + li.off[WS_DLIK];
    const uint8_t* ven = lb + li.off[WS_VEN];
    const uint8_t* vmin = lb + li.off[WS_VMIN];
    const uint8_t* dex = lb + li.off[WS_DEX];
    const void* xix = lb + li.off[WS_XOFF];
    const uint32_t* xloff = reinterpret_cast<const uint32_t*>(lb + li.off[WS_XLOFF]);
    const uint16_t* xids = reinterpret_cast<const uint16_t*>(lb + li.off[WS_XIDS]);
    const uint32_t* tokoff = reinterpret_cast<const uint32_t*>(lb + li.off[WS_TOKOFF]);
    const void* rix = lb + li.off[WS_ROFF];
    const uint32_t* rloff = reinterpret_cast<const uint32_t*>(lb + li.off[WS_RLOFF]);
    const uint16_t* rids = reinterpret_cast<const uint16_t*>(lb + li.off[WS_RIDS]);
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= B.n_utt) return;
    if (fbase[B.n_utt] > fcap) {                  // findings arena too small: re-run with the exact size
        if (u == 0) atomicOr(err, (uint32_t)ERR_QUEUE);
        return;
    }
    const WinIt it = win_begin(W, B, u);
    const int nw = it.nw;
    uint32_t WL = 0;
    for (int j = 0; j < nw; ++j) WL += win_at(W, B, it, j).len + 1;
    WL -= 1;
    const int T = R.T;
    const int g = win_ctx[u];
    const int v = g >= 0 ? g + 1 : 0;
    const int minlik = vmin[v];
    pii_span* fdu = wfd + fbase[u];
    uint32_t nf = 0;
    int delta = 0;
    uint32_t max_end = 0;
    uint32_t oj = 0;
    for (int j = 0; j < nw; ++j) {
        const WEntry Ej = win_at(W, B, it, j);
        int ex_s[NE_MAX], ex_e[NE_MAX], ex_t[NE_MAX];
        uint32_t ex_valid = 0;
        int s = -1, best_e = -1, best_t = 0, best_lik = 0;
        auto flush_start = [&]() {
            if (best_e >= 0 && oj + (uint32_t)s >= max_end) {
                pii_span f;
                f.utt = u;
                f.start = oj + (uint32_t)s;
                f.end = oj + (uint32_t)best_e;
                f.info_type = (uint16_t)best_t;
                f.likelihood = (uint8_t)best_lik;
                f.flags = 0;
                fdu[nf++] = f;
                max_end = f.end;
                delta += (int)(tokoff[best_t + 1] - tokoff[best_t]) - (best_e - s);
            }
            best_e = -1;
        };
        for (uint32_t k = 0; k < Ej.nc; ++k) {
            const WCand C = Ej.c[k];
            const int cs = (int)C.s, e = (int)C.e;
            if (cs != s) {
                flush_start();
                s = cs;
            }
            const int p = C.p;
            const int t = dtype[p];
            if (!ven[v * T + t]) continue;
            int lik = dlik[p];
            uint32_t r0, r1;
            list_range<true>(rix, li.aux & 7u, rloff, (uint32_t)(v * T + t), r0, r1);
            // resident proximity bits: at the window start the clipped ones, with >= need predecessors
            // the ones over the halo; otherwise (or for rules past WHOT_BITS) re-run over the window
            const bool known = C.need == 0 || j == 0 || j >= (int)C.need;
            const uint32_t bits = (C.need == 0 || j == 0) ? C.hot : C.hotx;
            for (uint32_t q = r0; q < r1; ++q) {
                const int h = rids[q];
                const int wb = hrule[4 * h], wa = hrule[4 * h + 1];
                const bool ca = wa > 0 && (uint32_t)(e + wa) > Ej.len && j + 1 < nw;   // reaches the next utterance
                const uint32_t ps = oj + (uint32_t)s, pe = oj + (uint32_t)e;
                bool hit;
                if (h < WHOT_BITS && known) {
                    hit = (bits >> h) & 1u;
                    if (!hit && ca) hit = hot_run_win(pool, hdesc + 8 * h, W, B, it, pe, min(WL, pe + (uint32_t)wa));
                } else {
                    hit = wb > 0 && hot_run_win(pool, hdesc + 8 * h, W, B, it, ps > (uint32_t)wb ? ps - wb : 0u, ps);
                    if (!hit && wa > 0) hit = hot_run_win(pool, hdesc + 8 * h, W, B, it, pe, min(WL, pe + (uint32_t)wa));
                }
                if (hit) {
                    const int fixed = hrule[4 * h + 2], rel = hrule[4 * h + 3];
                    if (fixed) {
                        lik = fixed;
                    } else {
                        lik += rel;
                        lik = lik < 1 ? 1 : (lik > 5 ? 5 : lik);
                    }
                }
            }
            const int xi = dex[p];
            if (lik < minlik) {
                if (xi != 0xff) ex_valid &= ~(1u << xi);
                continue;
            }
            if (xi != 0xff) {
#pragma unroll
                for (int x = 0; x < NE_MAX; ++x)
                    if (x == xi) {
                        ex_s[x] = s;
                        ex_e[x] = e;
                        ex_t[x] = t;
                    }
                ex_valid |= 1u << xi;
            }
            uint32_t x0, x1;
            list_range<true>(xix, (li.aux >> 3) & 7u, xloff, (uint32_t)(v * T + t), x0, x1);
            bool excluded = false;
            for (uint32_t q = x0; q < x1; ++q) {
                const int xt = xids[q];
#pragma unroll
                for (int x = 0; x < NE_MAX; ++x)
                    if (x != xi && ((ex_valid >> x) & 1) && ex_t[x] == xt && ex_s[x] <= s && e <= ex_e[x])
                        excluded = true;
            }
            if (excluded) continue;
            const bool better = best_e < 0 || e > best_e ||
                                (e == best_e && (lik > best_lik || (lik == best_lik && t < best_t)));
            if (better) {
                best_e = e;
                best_t = t;
                best_lik = lik;
            }
        }
        flush_start();
        oj += Ej.len + 1;
    }
    n_wfind[u] = nf;
    wout_len[u] = (uint32_t)((int)WL + delta);
}

// per conversation run (its last row): place the run's newest min(N, run) rows in the history ring.
// Entries are contiguous in the slot's arena (wrap to 0 when the tail is short); the final live set
// must not overlap, else ERR_RING (raise slot_bytes).  Nothing is written to the ring here.
__global__ __launch_bounds__(256) void k_win_alloc(const WinRing W, const WinBatch B, WNew* __restrict__ wnew,
                                                   uint32_t* __restrict__ err) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= B.n_utt || (*err & (ERR_ABORT | ERR_SLOT))) return;
    const uint32_t sl = B.slot[u];
    if (sl >= W.n_slots || (u + 1 < B.n_utt && B.slot[u + 1] == sl)) return;
    uint32_t k = 1;
    while (k < W.N && u >= k && B.slot[u - k] == sl) ++k;
    const uint32_t cnt = W.cnt[sl], head = W.head[sl], N = W.N, cap = W.slot_bytes;
    const uint32_t keep = min(cnt, N - k);                 // old entries that stay live
    uint32_t lo[WN_MAX], hi[WN_MAX];
    int nl = 0;
    uint32_t end = 0;
    for (uint32_t i = 0; i < cnt; ++i) {                    // oldest live .. newest
        const WDesc D = W.desc[(size_t)sl * N + (head + N - cnt + i) % N];
        end = D.off + 16u * D.nc + ((D.len + 15u) & ~15u);
        if (i >= cnt - keep) {
            lo[nl] = D.off;
            hi[nl] = end;
            ++nl;
        }
    }
    bool bad = false;
    for (uint32_t i = 0; i < k; ++i) {
        const uint32_t v = u - k + 1 + i;
        const uint64_t size = 16ull * B.wc_n[v] + ((B.offs[v + 1] - B.offs[v] + 15) & ~15ull);
        if (size > cap) {
            bad = true;
            break;
        }
        uint32_t pos = end;
        if ((uint64_t)pos + size > cap) pos = 0;
        for (int q = 0; q < nl; ++q)
            if (pos < hi[q] && lo[q] < pos + (uint32_t)size) bad = true;
        lo[nl] = pos;
        hi[nl] = pos + (uint32_t)size;
        ++nl;
        end = pos + (uint32_t)size;
        WNew w;
        w.off = pos;
        w.ri = (head + i) % N;
        w.cnt = min(N, cnt + k);
        w.head = (head + k) % N;
        wnew[v] = w;
    }
    if (bad) atomicOr(err, (uint32_t)ERR_RING);
}

// window output byte `rel` (slow path for windows whose pieces overflow the tile's LDS table)
__device__ uint8_t win_byte_slow(const RulesDev& R, const WinRing& W, const WinBatch& B, const WinIt& it,
                                 const pii_span* F, uint32_t nf, uint32_t rel) {
    uint32_t pout = 0, fi = 0, oj = 0;
    for (int j = 0; j < it.nw; ++j) {
        const WEntry Ej = win_at(W, B, it, j);
        const uint32_t sh = oj + Ej.len;
        uint32_t pin = oj;
        while (fi < nf && F[fi].start < sh) {
            const uint32_t run = F[fi].start - pin;
            if (rel < pout + run) return Ej.t[pin - oj + (rel - pout)];
            pout += run;
            const uint32_t t0 = R.tok_off[F[fi].info_type], tl = R.tok_off[F[fi].info_type + 1] - t0;
            if (rel < pout + tl) return R.tok_bytes[t0 + (rel - pout)];
            pout += tl;
            pin = F[fi].end;
            ++fi;
        }
        const uint32_t run = sh - pin;
        if (rel < pout + run) return Ej.t[pin - oj + (rel - pout)];
        pout += run;
        if (rel == pout) return '\n';
        ++pout;
        oj = sh + 1;
    }
    return 0;
}

// WIN_TILE windows per workgroup: piece table (copy runs of each resident / batch utterance, tokens,
// '\n' separators) in LDS, then the shared 16-byte block assembly; spans copied out
__global__ __launch_bounds__(REDACT_BLOCK) void k_win_redact(const RulesDev R, const WinRing W, const WinBatch B,
                                                             const pii_span* __restrict__ wfd,
                                                             const uint64_t* __restrict__ fbase,
                                                             const uint32_t* __restrict__ n_wfind,
                                                             const uint64_t* __restrict__ out_offs,
                                                             const uint64_t* __restrict__ span_offs,
                                                             const uint32_t* __restrict__ err, uint8_t* __restrict__ out,
                                                             pii_span* __restrict__ spans) {
    __shared__ uint32_t s_pout[PIECE_MAX + 1];
    __shared__ uint64_t s_psrc[PIECE_MAX + 1];
    __shared__ uint32_t s_wsum[REDACT_BLOCK / 64];
    __shared__ uint16_t s_bp[BLK_MAX];
    __shared__ uint32_t s_total;
    if (*err != 0) return;
    const uint32_t u0 = blockIdx.x * WIN_TILE;
    const uint32_t u1 = min(u0 + WIN_TILE, B.n_utt);
    const uint32_t nu = u1 - u0;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t out_lo = (int64_t)out_offs[u0], out_hi = (int64_t)out_offs[u1];
    const bool mine = (uint32_t)tid < nu;        // WIN_TILE == 64: wavefront 0 owns the windows
    const uint32_t u = u0 + tid;
    WinIt it;
    it.nw = 0;
    uint32_t nf = 0;
    if (mine) {
        it = win_begin(W, B, u);
        nf = n_wfind[u];
    }
    const uint32_t cnt = mine ? 2 * nf + 2 * (uint32_t)it.nw - 1 : 0;
    uint32_t incl = cnt;
    if (wid == 0) {
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(incl, d);
            if (lane >= d) incl += x;
        }
        if (lane == 63) s_total = incl;
    }
    __syncthreads();
    const uint32_t total_p = s_total;
    const bool staged = total_p <= PIECE_MAX;
    if (mine) {
        const pii_span* F = wfd + fbase[u];
        pii_span* sp = spans + span_offs[u];
        for (uint32_t f = 0; f < nf; ++f) sp[f] = F[f];
        if (staged) {
            uint32_t pb = incl - cnt;
            uint32_t po = (uint32_t)((int64_t)out_offs[u] - out_lo);
            uint32_t fi = 0, oj = 0;
            for (int j = 0; j < it.nw; ++j) {
                const WEntry Ej = win_at(W, B, it, j);
                const uint32_t sh = oj + Ej.len;
                const uint64_t src = (uint64_t)(uintptr_t)Ej.t - oj;     // window position -> address
                uint32_t pin = oj;
                while (fi < nf && F[fi].start < sh) {
                    const pii_span Fi = F[fi];
                    s_pout[pb] = po;
                    s_psrc[pb] = src + pin;
                    ++pb;
                    po += Fi.start - pin;
                    const uint32_t t0 = R.tok_off[Fi.info_type];
                    s_pout[pb] = po;
                    s_psrc[pb] = (uint64_t)(uintptr_t)(R.tok_bytes + t0);
                    ++pb;
                    po += R.tok_off[Fi.info_type + 1] - t0;
                    pin = Fi.end;
                    ++fi;
                }
                s_pout[pb] = po;
                s_psrc[pb] = src + pin;
                ++pb;
                po += sh - pin;
                if (j + 1 < it.nw) {
                    s_pout[pb] = po;
                    s_psrc[pb] = (uint64_t)(uintptr_t)(R.tok_bytes + R.nl_off);
                    ++pb;
                    po += 1;
                }
                oj = sh + 1;
            }
        }
    }
    if (tid == 0 && staged) s_pout[total_p] = (uint32_t)(out_hi - out_lo);
    __syncthreads();
    if (staged) {
        tile_assemble<false>(s_pout, s_psrc, total_p, s_bp, s_wsum, out, out_lo, out_hi);
    } else {
        // one wavefront per window, byte-granular
        for (uint32_t i = wid; i < nu; i += REDACT_BLOCK / 64) {
            const uint32_t uu = u0 + i;
            const WinIt iu = win_begin(W, B, uu);
            const pii_span* F = wfd + fbase[uu];
            const uint32_t nfi = n_wfind[uu];
            uint8_t* dst = out + out_offs[uu];
            const uint32_t olen = (uint32_t)(out_offs[uu + 1] - out_offs[uu]);
            for (uint32_t rel = lane; rel < olen; rel += 64) dst[rel] = win_byte_slow(R, W, B, iu, F, nfi, rel);
        }
    }
}

// after a successful call: the planned rows enter the rings (16 threads per row copy the resident
// candidates, then the text, as aligned 16-byte stores); descriptors, counts and heads follow
__global__ __launch_bounds__(256) void k_win_commit(const WinRing W, const WinBatch B, const WNew* __restrict__ wnew,
                                                    const uint32_t* __restrict__ err) {
    if (*err != 0) return;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t v = (uint32_t)(gid >> 4), t = (uint32_t)(gid & 15);
    if (v >= B.n_utt) return;
    const WNew w = wnew[v];
    if (w.off == 0xffffffffu) return;
    const uint32_t sl = B.slot[v];
    const uint32_t nc = B.wc_n[v];
    const uint64_t a = B.offs[v];
    const uint32_t len = (uint32_t)(B.offs[v + 1] - a);
    uint8_t* dst = W.arena + (size_t)sl * W.slot_bytes + w.off;
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    if (nc) {
        const uint4* c4 = reinterpret_cast<const uint4*>(B.wc + B.wc_first[v]);
        for (uint32_t k = t; k < nc; k += 16) d4[k] = c4[k];
    }
    const uint8_t* src = B.text + a;
    for (uint32_t q = t; 16 * q < len; q += 16) {
        const int n = len - 16 * q < 16 ? (int)(len - 16 * q) : 16;
        d4[nc + q] = load16(src + 16 * q, 0, n);
    }
    if (t == 0) {
        WDesc D;
        D.off = w.off;
        D.len = len;
        D.nc = nc;
        D.pad = 0;
        W.desc[(size_t)sl * W.N + w.ri] = D;
        const bool last = v + 1 == B.n_utt || B.slot[v + 1] != sl;
        if (last) {
            W.cnt[sl] = w.cnt;
            W.head[sl] = w.head;
        }
    }
}

// ---- full re-scan of the joined windows (rule sets the incremental path cannot take: a detector that
// consumes '\n' or tests a text edge, several SCAN groups, tables past LDS).  The ring then holds the
// raw text only (no resident candidates, wc_n = 0); each row's window "\n".join(ring entries, batch
// predecessors, row) is materialised in HBM and run through the ordinary pipeline as one row.
// per row: its joined window's length
__global__ __launch_bounds__(256) void k_win_jlen(const WinRing W, const WinBatch B, uint32_t* __restrict__ jlen,
                                                  const uint32_t* __restrict__ err) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= B.n_utt) return;
    if (*err & (ERR_ABORT | ERR_SLOT)) {
        jlen[u] = 0;
        return;
    }
    const WinIt it = win_begin(W, B, u);
    uint32_t n = (uint32_t)it.nw - 1u;
    for (int j = 0; j < it.nw; ++j) n += win_at(W, B, it, j).len;
    jlen[u] = n;
}

// one wavefront per row: copy its window's entries and the '\n' joins to jbuf + joff[u]
__global__ __launch_bounds__(256) void k_win_join(const WinRing W, const WinBatch B, const uint64_t* __restrict__ joff,
                                                  uint8_t* __restrict__ jbuf, const uint32_t* __restrict__ err) {
    const uint32_t u = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (u >= B.n_utt || (*err & (ERR_ABORT | ERR_SLOT))) return;
    const WinIt it = win_begin(W, B, u);
    uint64_t pos = joff[u];
    for (int j = 0; j < it.nw; ++j) {
        const WEntry E = win_at(W, B, it, j);
        for (uint32_t k = lane; k < E.len; k += 64) jbuf[pos + k] = E.t[k];
        pos += E.len;
        if (j + 1 < it.nw) {
            if (lane == 0) jbuf[pos] = '\n';
            ++pos;
        }
    }
}

// the counter block a second pass over the same call starts from: the first pass's error flags and its
// context commit count.  The first pass writes no pair queue (launch_front with pair_first = false), so
// an ERR_QUEUE here is a real overflow: it is kept, with the queue needs, so that every stage of pass 2
// bails out and pii_sync grows the queues and re-runs the call.
__global__ void k_err_save(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ saved) {
    saved[0] = cnt[0];
    saved[1] = 0;
    saved[2] = cnt[2];
    saved[3] = cnt[3];
    saved[4] = cnt[4];
    saved[5] = cnt[5];
}

// the totals of a context-only call (pii_context_update): no output, no spans, its error flags
__global__ void k_ctx_totals(const uint32_t* __restrict__ err, uint64_t* __restrict__ totals) {
    totals[0] = totals[1] = 0;
    totals[2] = *err;
    totals[3] = totals[4] = totals[5] = 0;
}

// a call's first kernel: its counter block (err, long_count, ncommit, pair_count) from zero or from a
// first pass's block, the lane-sort buckets, and a histogram reset deferred to here (three memset /
// copy commands were ~15 us of gaps per call)
__global__ __launch_bounds__(256) void k_begin(uint32_t* __restrict__ d_err, const uint32_t* __restrict__ err_init,
                                               uint32_t* __restrict__ lane_bkt, uint32_t nbkt,
                                               unsigned long long* __restrict__ hist, uint32_t nhist) {
    const uint32_t t = threadIdx.x;
    if (t < 6) d_err[t] = err_init ? err_init[t] : 0u;
    for (uint32_t i = t; i < nbkt; i += blockDim.x) lane_bkt[i] = 0;
    for (uint32_t i = t; i < nhist; i += blockDim.x) hist[i] = 0;
}

__global__ void k_noop() {}

// ------------------------------------------------------------------------------- LDS images
// DFAs re-packed into a kernel's own pool (descriptor offsets rebased; each transition entry carries
// the destination's flags in bits 14-15, see pii_device.h)
struct DfaPool {
    std::vector<uint16_t> trans;
    std::vector<uint8_t> cmap;
    std::vector<int32_t> desc;
};
bool add_dfa(DfaPool& dp, const int32_t* d, const uint16_t* trans, const uint8_t* flags, const uint8_t* cmap) {
    const int32_t nc = d[3], ns = d[7];
    if (ns > (int32_t)DFA_STATE_MASK + 1) return false;
    int32_t nd[8];
    std::memcpy(nd, d, sizeof(nd));
    // LDS bank stagger (32 banks x 4 B): a pair kernel's wavefront runs many patterns' automata over
    // the same text bytes, so automaton k's transition table starts at bank k mod 32 and its class map
    // 4 bytes after the previous map's end (byte c of every map would otherwise sit in one bank)
    const size_t k = dp.desc.size() / 8;
    while (dp.trans.size() % 64 != (2 * k) % 64) dp.trans.push_back(0);
    nd[0] = (int32_t)dp.trans.size();
    nd[1] = 0;
    nd[2] = (int32_t)dp.cmap.size();
    for (size_t i = 0; i < (size_t)ns * nc; ++i) {
        const uint16_t dst = trans[d[0] + i];
        dp.trans.push_back((uint16_t)(dst | ((flags[d[1] + dst] & 3u) << 14)));
    }
    dp.cmap.insert(dp.cmap.end(), cmap + d[2], cmap + d[2] + 256);
    dp.cmap.insert(dp.cmap.end(), 4, (uint8_t)0);
    dp.desc.insert(dp.desc.end(), nd, nd + 8);
    return true;
}

// ------------------------------------------------------------------------------- blob parsing
struct Section {
    std::string name;
    uint32_t dtype;
    const uint8_t* data;
    uint64_t bytes;
};

bool parse_blob(const uint8_t* p, size_t n, std::vector<Section>& out) {
    if (n < 12 || std::memcmp(p, "PIIRULE1", 8) != 0) return false;
    uint32_t cnt;
    std::memcpy(&cnt, p + 8, 4);
    size_t off = 12;
    for (uint32_t i = 0; i < cnt; ++i) {
        uint32_t ln;
        if (off + 4 > n) return false;
        std::memcpy(&ln, p + off, 4);
        off += 4;
        if (off + ln + 12 > n) return false;
        Section s;
        s.name.assign(reinterpret_cast<const char*>(p + off), ln);
        off += ln;
        std::memcpy(&s.dtype, p + off, 4);
        std::memcpy(&s.bytes, p + off + 4, 8);
        off += 12;
        if (off + s.bytes > n) return false;
        s.data = p + off;
        off += s.bytes;
        off += (8 - off % 8) % 8;
        out.push_back(s);
    }
    return true;
}

}  // namespace

// ================================================================================ engine object
constexpr size_t IMG_LDS_MAX = 160 * 1024;
// k_pair_first<true>'s LDS copy: most of the LDS, one 1024-thread workgroup per CU (config 5: 40 / 78 /
// 156 KB -> 999 / 934 / 885 us: more automata in LDS beat two workgroups per CU)
constexpr size_t FIRST_HOT_LDS = 156 * 1024;
constexpr size_t FIRST_HOT_BIG = 8 * 1024;      // ... which skips automata larger than this (prefix of
                                                // ids, 78 KB: 982 -> 933 us)
constexpr size_t IMG_LDS_SPLIT = 80 * 1024;    // pair-kernel image size past which its per-(variant, type) lists stay in L2
struct DevImage {
    LdsImage li{};
    uint4* d = nullptr;
    bool global = false;      // larger than LDS: kernels read it in place (load_image<true>)
    size_t lds() const { return global ? 0 : li.total; }
};

// a per-(variant, type) list table, deduplicated for the LDS images (list_range)
struct ListTab {
    std::vector<uint8_t> ix;      // per key: list number, w bytes
    std::vector<uint32_t> loff;   // per list: first id, + end
    std::vector<uint16_t> ids;
    uint32_t w = 1;
};
// (a small table stays as it is -- w = 0, ix empty: one LDS read less per lookup; config 2's list
// lookups in k_select cost 4 us more through the index)
constexpr size_t LIST_DEDUP_KEYS = 8192;
static ListTab dedup_lists(const uint32_t* off, const uint16_t* ids, size_t n_keys) {
    ListTab t;
    if (n_keys <= LIST_DEDUP_KEYS) {
        t.w = 0;
        t.ix.push_back(0);
        t.loff.assign(off, off + n_keys + 1);
        t.ids.assign(ids, ids + off[n_keys]);
        if (t.ids.empty()) t.ids.push_back(0);
        return t;
    }
    std::map<std::vector<uint16_t>, uint32_t> uniq;
    std::vector<uint32_t> num(n_keys);
    t.loff.push_back(0);
    for (size_t i = 0; i < n_keys; ++i) {
        std::vector<uint16_t> l(ids + off[i], ids + off[i + 1]);
        auto it = uniq.find(l);
        if (it == uniq.end()) {
            it = uniq.emplace(l, (uint32_t)uniq.size()).first;
            t.ids.insert(t.ids.end(), l.begin(), l.end());
            t.loff.push_back((uint32_t)t.ids.size());
        }
        num[i] = it->second;
    }
    const size_t n = uniq.size();
    t.w = n <= 256 ? 1u : (n <= 65536 ? 2u : 4u);
    t.ix.resize(n_keys * t.w);
    for (size_t i = 0; i < n_keys; ++i) std::memcpy(t.ix.data() + i * t.w, &num[i], t.w);   // little endian
    if (t.ids.empty()) t.ids.push_back(0);
    return t;
}

// packs `parts` (16-byte aligned sections) into one image and uploads it
static bool make_image(const std::vector<std::pair<const void*, size_t>>& parts, DevImage& out) {
    if (parts.size() > (size_t)IMG_MAX) return false;
    size_t off = 0;
    for (size_t i = 0; i < parts.size(); ++i) {
        out.li.off[i] = (uint32_t)off;
        off += (parts[i].second + 15) & ~(size_t)15;
    }
    if (off == 0) off = 16;
    out.li.total = (uint32_t)off;
    out.global = off > IMG_LDS_MAX;
    std::vector<uint8_t> img(off, 0);
    for (size_t i = 0; i < parts.size(); ++i)
        if (parts[i].second) std::memcpy(img.data() + out.li.off[i], parts[i].first, parts[i].second);
    return hipMalloc(reinterpret_cast<void**>(&out.d), off) == hipSuccess &&
           hipMemcpy(out.d, img.data(), off, hipMemcpyHostToDevice) == hipSuccess;
}

struct pii_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    RulesDev R{};
    void* d_rules = nullptr;
    std::vector<std::string> names;
    std::vector<int> kw_type;
    uint32_t n_slots = 0;
    int64_t ttl_us = 0;
    size_t scan_lds = 0;
    // SCAN groups (config-5 scale rule sets: one reverse D automaton per k_scan pass; sg[0] = R)
    uint32_t n_sg = 1;
    std::vector<RulesDev> sg;
    std::vector<size_t> sg_lds;
    RulesDev* d_sg = nullptr;          // sg and sg_lds in device memory (k_scan_fix, all groups at once)
    uint32_t* d_sg_lds = nullptr;
    size_t max_sg_lds = 0;
    AccTabs acct{};
    uint32_t* lane_evn = nullptr;      // per lane: events of all groups (k_pairs_merge)
    DevImage img_first, img_eval, img_sel, img_wsel;     // per-kernel LDS images of the rule tables
    DevImage img_first_hot;            // img_first past LDS: the automata of its first first_p_hot patterns
    uint32_t first_p_hot = 0;
    bool lists_cl = false;
    hipStream_t aux[2] = {nullptr, nullptr};   // more streams for the SCAN groups' passes (PII_SCAN_STREAMS)
    uint32_t n_aux = 0;
    hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};             // the images' rule / exclusion lists are deduplicated (list_range)
    DevImage img_eval_rg;     // k_pair_eval's image without the rule lists (built when img_eval is past IMG_LDS_SPLIT)
    DevImage img_sel_rg;      // k_select's image without the exclusion lists (likewise)
    int n_cu = 256;
    // persistent state (replaces Redis)
    int32_t* st_group = nullptr;
    int64_t* st_ts = nullptr;
    uint32_t* stamp = nullptr;
    uint32_t epoch = 0;
    unsigned long long* hist = nullptr;
    uint32_t* hist_part = nullptr;     // per redact tile, per info type
    // scratch
    uint64_t cap_bytes = 0, cap_lanes = 0;
    uint32_t lane_shift = 10, last_lanes = 0;     // scan lane = utterances starting in 2^lane_shift bytes
    uint32_t cap_utt = 0;
    size_t cap_bsum = 0;
    Event* ev = nullptr;
    pii_span* fd = nullptr;
    uint32_t *n_ev = nullptr, *n_find = nullptr, *out_len = nullptr, *incl = nullptr, *agg_f = nullptr;
    uint32_t* first_utt = nullptr;
    uint4* lane_geo = nullptr;         // per lane geometry (Geo::lanes)
    uint32_t* lane_perm = nullptr;     // k_scan slot -> lane (longest lanes first)
    uint32_t* lane_pos = nullptr;      // lane -> slot
    uint32_t* lane_bkt = nullptr;      // [2 * LANE_NB] bucket counts + reservation cursors
    uint32_t* lane_cnt = nullptr;
    uint64_t* bnd = nullptr;
    uint32_t* lane_split = nullptr;    // k_scan2: per slot split point | A's arena capacity (k_lane_bits2)
    uint32_t* lane_spl = nullptr;      // the same per lane (k_lane_count)
    bool scan2 = false;                // two chains per lane in the SCAN (PII_SCAN2=1: k_scan2; slower)
    uint32_t halo_items = HALO_ITEMS;  // k_win_halo's item list per workgroup (PII_HALO_ITEMS: tests)
    bool scan_ilv = true;              // k_scan grids of <= n_cu workgroups deal wavefronts round-robin (PII_SCAN_ILV)
    uint32_t win_long = 0;             // incremental re-scan: rows longer than this many lanes are cut (PII_WIN_LONG; 0: never)
    EvLoc* evloc = nullptr;
    uint64_t ev_cap = 0;
    uint64_t* lane_ev = nullptr;      // exclusive scan of lane_cnt: first dense event index per lane
    PairRes* pres = nullptr;
    int32_t* pend = nullptr;          // FIRST end per pair
    uint64_t pair_cap = 0;
    unsigned long long* pair_count = nullptr;
    uint64_t* lane_pair = nullptr;
    uint32_t* lane_np = nullptr;
    uint32_t* matched = nullptr;
    uint32_t* mcount = nullptr;   // matched pairs per k_pair_first wavefront segment
    FirstCont* cont = nullptr;
    uint32_t n_seg = 0;
    uint32_t eval_split = 2;           // k_pair_eval work units per k_pair_first workgroup (PII_EVAL_SPLIT)
    uint32_t merge_cap = MERGE_EVW;    // k_pairs_merge: events a wavefront stages (PII_MERGE_CAP; 0: walk)
    struct Call {
        const uint8_t* text;
        const uint64_t* offs;
        uint32_t n_utt;
        uint64_t base;
        uint64_t total;
        const uint32_t* slot;
        const uint8_t* role;
        const int64_t* ts;
        uint8_t* out;
        uint64_t out_cap;
        uint64_t* out_offs;
        pii_span* spans;
        uint32_t span_cap;
        int16_t* ctx_info;
        hipStream_t st;
        const pii_span* ext;
        const uint32_t* ext_n;
        uint32_t ext_stride;
    } last{};
    int32_t* kw = nullptr;
    int16_t* ctx = nullptr;
    int32_t *agg_v = nullptr, *commit = nullptr;
    uint64_t *span_offs = nullptr, *bsum = nullptr, *out_offs_tmp = nullptr;
    unsigned long long *lb_state = nullptr, *lb_ticket = nullptr;   // single-pass scan tiles / ticket counter
    uint32_t lb_cap = 0, lb_epoch = 0;
    uint32_t* d_err = nullptr;            // counter block (one memset per call): err, long_count, ncommit, pair_count
    uint32_t* ncommit = nullptr;          // k_ctx_apply's commit-list length
    uint64_t* d_totals = nullptr;
    uint64_t* h_totals = nullptr;    // pinned copy of d_totals (+ the histogram behind it)
    bool h_hist_valid = false;       // h_totals' histogram is the device's as of the last call (no reset since)
    bool hist_zero_pending = false;  // pii_histogram_reset since the last call: its k_begin zeroes the histogram
    // host-API staging
    uint64_t cap_h_bytes = 0, cap_h_out = 0;
    uint32_t cap_h_utt = 0, cap_h_spans = 0;
    uint8_t *h_text = nullptr, *h_role = nullptr, *h_out = nullptr;
    uint64_t *h_offs = nullptr, *h_out_offs = nullptr;
    uint32_t* h_slot = nullptr;
    int64_t* h_ts = nullptr;
    pii_span* h_spans = nullptr;
    int16_t* h_ctx = nullptr;
    pii_span* h_ext = nullptr;         // external candidates of a host-buffer call
    uint32_t* h_ext_n = nullptr;
    uint64_t cap_h_ext = 0;
    uint32_t cap_h_ext_n = 0;
    hipEvent_t tev[7] = {};
    // what a call records with HIP events (pii_set_timing): 0 = only the completion event; 1 = + the
    // call's start and the events around k_scan / k_redact (the roofline kernels); 2 = + the stage
    // boundaries (pii_last_timings [0..4]).  An event record between two kernels costs ~6 us of GPU
    // time (the queue drains at the marker): level 2's five stage events were ~30 us of a config-2
    // step and ~12% of a window re-scan step (rocprofv3 kernel trace gaps).
    int timing = 1;
    float last_ms[6] = {};
    hipEvent_t kev[4] = {};           // around k_scan and k_redact (the roofline kernels)
    bool kev_valid = false;
    float last_kms[2] = {};
    int last_kind = 0;                // 0 = pii_scan_redact*, 1 = pii_rescan_window* (what pii_sync re-runs)
    // window re-scan (a12): resident history rings + per-call scratch
    uint32_t win_n = 0, win_slot_bytes = 0;
    bool window_ok = false;
    WDesc* wr_desc = nullptr;
    uint32_t *wr_cnt = nullptr, *wr_head = nullptr;
    uint8_t* wr_arena = nullptr;
    WCand* wc = nullptr;
    uint32_t* phot = nullptr;
    uint64_t wc_cap = 0;
    uint32_t *wc_first = nullptr, *wc_n = nullptr, *wbound = nullptr, *n_wfind = nullptr, *wout_len = nullptr;
    uint64_t *wfbase = nullptr, *wspan_offs = nullptr;
    WNew* wnew = nullptr;
    int16_t* wctx = nullptr;
    uint32_t wcap_utt = 0;
    pii_span* wfd = nullptr;
    uint64_t wfd_cap = 0;
    // full window re-scan (win_full): joined windows, their offsets, a second keyword array, all-CUSTOMER
    // roles and the first pass's counter block
    bool win_full = false;
    uint8_t* jbuf = nullptr;
    uint64_t cap_jbuf = 0;
    uint64_t* joff = nullptr;
    uint32_t* jlen = nullptr;
    int32_t* kw2 = nullptr;
    uint8_t* jrole = nullptr;
    uint32_t cap_j_utt = 0;
    uint32_t* err_saved = nullptr;
    uint64_t* h_jtotal = nullptr;      // pinned: the joined bytes of the call
    // work-buffer accounting (grow): bytes per buffer, their sum, the limit (0 = none)
    std::unordered_map<void*, size_t> scratch_sizes;
    uint64_t scratch_used = 0, scratch_limit = 0;
    // lane-based resolve, long rows, span-driven redaction
    uint32_t r0 = 0, long_min = NO_CUTS;
    uint32_t* long_rows = nullptr;     // rows cut into several lanes (k_chunk_index)
    uint32_t* long_count = nullptr;
    uint64_t cap_long = 0, cap_ev = 0, cap_fd = 0;
    uint32_t* lane_st = nullptr;       // [2 * lanes] scan state handed across cuts (k_scan_fix)
    uint32_t* lane_nf = nullptr;       // findings per lane
    int2* lane_rd = nullptr;           // cut-row deltas per lane
    uint32_t* lane_reach = nullptr;
    int32_t* lane_rowbase = nullptr;
    uint8_t* dirty = nullptr;
    uint64_t* lane_sp = nullptr;       // exclusive scan of lane_nf (span offsets); [lanes] = total spans
    uint2* spill = nullptr;            // k_select's per-run (pattern, end) lists, indexed like the pair queue
    RSpan* rsp = nullptr;
    uint64_t cap_rsp = 0;
    uint32_t* tile_first = nullptr;
    uint64_t cap_tiles = 0;
    uint32_t hist_types = 0;           // types counted per workgroup in LDS (k_spans)
};

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t _e = (x);                                                       \
        if (_e != hipSuccess) {                                                    \
            e->err = std::string(#x) + ": " + hipGetErrorString(_e);              \
            return PII_E_DEVICE;                                                   \
        }                                                                          \
    } while (0)

namespace {

// (Re)size a work buffer.  The new buffer is allocated before the old one is freed, so a failure
// leaves the old buffer -- and the capacity the caller recorded for it -- intact; the engine stays
// usable for calls that fit.  Work buffers count against the scratch limit (pii_set_scratch_limit).
template <class T>
int grow(pii_engine* e, T*& p, size_t count) {
    if (count == 0) count = 1;
    const size_t nb = count * sizeof(T);
    size_t old = 0;
    if (p) {
        auto it = e->scratch_sizes.find(static_cast<void*>(p));
        if (it != e->scratch_sizes.end()) old = it->second;
    }
    if (e->scratch_limit && e->scratch_used - old + nb > e->scratch_limit) {
        e->err = "device allocation failed: the engine's work buffers would exceed its scratch limit";
        return PII_E_NOMEM;
    }
    T* q = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&q), nb) != hipSuccess) {
        (void)hipGetLastError();
        e->err = "device allocation failed";
        return PII_E_NOMEM;
    }
    if (p) {
        (void)hipFree(p);
        e->scratch_sizes.erase(static_cast<void*>(p));
        e->scratch_used -= old;
    }
    p = q;
    e->scratch_sizes[static_cast<void*>(q)] = nb;
    e->scratch_used += nb;
    return PII_OK;
}

int grow_pairs(pii_engine* e, uint64_t cap) {
    if (cap >= (1ull << 32)) {
        e->err = "pair queue beyond 2^32 entries; split the batch";
        return PII_E_NOMEM;
    }
    int rc;
    if ((rc = grow(e, e->pres, cap)) || (rc = grow(e, e->pend, cap + 16)) || (rc = grow(e, e->matched, cap)) ||
        (rc = grow(e, e->cont, cap)) || (rc = grow(e, e->spill, cap + 16)))
        return rc;
    return PII_OK;
}

int ensure_scratch(pii_engine* e, uint32_t n_utt, uint64_t bytes, uint32_t n_lanes, int min_len = 0) {
    int rc = PII_OK;
    // event arenas: a lane's emitted positions + its utterance starts (ev_base); findings arenas:
    // one finding per min_len bytes + one per lane (fd_base; min_len 1 when external spans come in)
    if (min_len <= 0) min_len = e->R.min_len;
    const uint64_t need_ev = bytes + n_utt + n_lanes + 2, need_fd = bytes / (uint64_t)min_len + n_lanes + 2;
    if (need_ev > e->cap_ev) {           // one arena per SCAN group, cap_ev events apart
        const uint64_t nb = std::max<uint64_t>(need_ev + need_ev / 8, 1 << 16);
        if ((rc = grow(e, e->ev, nb * e->n_sg))) return rc;
        e->cap_ev = nb;
    }
    if (need_fd > e->cap_fd) {
        const uint64_t nb = std::max<uint64_t>(need_fd + need_fd / 8, 1 << 12);
        if ((rc = grow(e, e->fd, nb))) return rc;
        e->cap_fd = nb;
    }
    if (bytes > e->cap_bytes) e->cap_bytes = bytes;
    if (n_lanes + 2 > e->cap_lanes) {
        const uint64_t nl = std::max<uint64_t>(n_lanes + n_lanes / 8 + 2, 1024);
        if ((rc = grow(e, e->first_utt, nl))) return rc;
        if ((rc = grow(e, e->lane_perm, nl))) return rc;
        if ((rc = grow(e, e->lane_pos, nl))) return rc;
        if ((rc = grow(e, e->lane_bkt, 2 * LANE_NB))) return rc;
        if ((rc = grow(e, e->lane_cnt, nl * e->n_sg))) return rc;
        if (e->n_sg > 1 && (rc = grow(e, e->lane_evn, nl))) return rc;
        if ((rc = grow(e, e->lane_ev, nl))) return rc;
        // utterance-start words: k_scan's u64 per block (LANE_WORDS rows) or k_scan2's u32 per
        // half-block (HB_A + HB_B rows), one buffer for either
        if ((rc = grow(e, e->bnd, nl * std::max<uint64_t>(LANE_WORDS, (HB_A + HB_B) / 2)))) return rc;
        if ((rc = grow(e, e->lane_split, nl))) return rc;
        if ((rc = grow(e, e->lane_spl, nl))) return rc;
        if ((rc = grow(e, e->lane_pair, nl))) return rc;
        if ((rc = grow(e, e->lane_np, nl))) return rc;
        if ((rc = grow(e, e->lane_st, 2 * nl * e->n_sg))) return rc;
        if ((rc = grow(e, e->lane_nf, nl))) return rc;
        if ((rc = grow(e, e->lane_rd, nl))) return rc;
        if ((rc = grow(e, e->lane_geo, nl))) return rc;
        if ((rc = grow(e, e->lane_reach, nl))) return rc;
        if ((rc = grow(e, e->lane_rowbase, nl))) return rc;
        if ((rc = grow(e, e->dirty, nl))) return rc;
        if ((rc = grow(e, e->lane_sp, nl + 1))) return rc;
        if ((rc = grow(e, e->hist_part, (nl / 256 + 2) * (size_t)std::max<uint32_t>(e->hist_types, 1)))) return rc;
        e->cap_lanes = nl;
        e->cap_bsum = 0;
    }
    // rows cut into lanes (k_chunk_index's long-row list): a long row is longer than long_min = 2 lanes,
    // and lanes shrink to 2^MIN_LANE_SHIFT bytes for small batches -- so at most bytes / 256 of them
    // (sizing this for 1 KiB lanes overflowed the list on a full window re-scan of 50k conversations,
    // whose ~600-byte joined windows are all long rows of 256-byte lanes)
    const uint64_t need_long = std::min<uint64_t>((uint64_t)n_utt + 1, bytes / (2u << MIN_LANE_SHIFT) + 2);
    if (need_long > e->cap_long) {
        if ((rc = grow(e, e->long_rows, need_long))) return rc;
        e->cap_long = need_long;
    }
    if (n_utt > e->cap_utt) {
        const uint32_t nu = std::max<uint32_t>(n_utt + n_utt / 8, 1024);
        if ((rc = grow(e, e->n_ev, nu))) return rc;
        if ((rc = grow(e, e->out_len, nu))) return rc;
        if ((rc = grow(e, e->incl, nu))) return rc;
        if ((rc = grow(e, e->kw, nu))) return rc;
        if ((rc = grow(e, e->ctx, nu))) return rc;
        if ((rc = grow(e, e->commit, nu))) return rc;
        const uint32_t nblk = nu / CTX_BLOCK + 2;
        if ((rc = grow(e, e->agg_v, nblk))) return rc;
        if ((rc = grow(e, e->agg_f, nblk))) return rc;
        e->cap_utt = nu;
        e->cap_bsum = 0;
    }
    if (e->cap_bsum == 0) {   // scan block sums: the utterance scans and the per-lane pair-count scan
        const size_t n = std::max<size_t>(e->cap_utt, e->cap_lanes);
        if ((rc = grow(e, e->bsum, 2 * (n / SCAN_TILE + 4)))) return rc;     // two scans per launch
        e->cap_bsum = n;
    }
    return rc;
}

// span list + output tiles for a call with these capacities
int ensure_redact(pii_engine* e, uint64_t span_cap, uint64_t out_cap) {
    int rc;
    if (span_cap + 1 > e->cap_rsp) {
        const uint64_t n = std::max<uint64_t>(span_cap + span_cap / 8 + 16, 4096);
        if ((rc = grow(e, e->rsp, n))) return rc;
        e->cap_rsp = n;
    }
    const uint64_t tiles = (out_cap >> RTILE_SHIFT) + 2;
    if (tiles > e->cap_tiles) {
        if ((rc = grow(e, e->tile_first, tiles + tiles / 8))) return rc;
        e->cap_tiles = tiles + tiles / 8;
    }
    return PII_OK;
}

// Small scans (a re-scan step: ~100k rows) take the single-pass look-back kernel, one launch instead
// of three; big ones (10M rows) the reduce / scan-of-sums / apply triple, whose tiles never wait on
// each other (the look-back's cross-XCD hand-offs chain up over thousands of tiles: 0.4 ms vs 0.06).
constexpr uint32_t LB_MAX_TILES = 64;

int exclusive_scan(pii_engine* e, const uint32_t* in, uint32_t n, uint64_t* out, hipStream_t st,
                   const uint32_t* in2 = nullptr, uint32_t n2 = 0, uint64_t* out2 = nullptr) {
    const uint32_t nb = (n + LB_TILE - 1) / LB_TILE, nb2 = in2 ? (n2 + LB_TILE - 1) / LB_TILE : 0;
    if (in2 == nullptr && nb == 0) {
        HIPCHK(hipMemsetAsync(out, 0, sizeof(uint64_t), st));
        return PII_OK;
    }
    // (a scan of zero items still writes its total: the look-back form needs a tile for it)
    if (nb > LB_MAX_TILES || nb2 > LB_MAX_TILES || (in2 && (nb == 0 || nb2 == 0))) {
        // reduce / scan-of-sums / apply; a second scan rides along in blockIdx.y
        ScanArgs a{{in, in2 ? in2 : in}, {out, out2 ? out2 : out}, {n, in2 ? n2 : 0u}, 0};
        const uint32_t nt = std::max<uint32_t>(1, (std::max(n, a.n[1]) + SCAN_TILE - 1) / SCAN_TILE);
        a.bstride = nt + 2;
        const uint32_t ny = in2 ? 2 : 1;
        k_scan_reduce<<<dim3(nt, ny), 256, 0, st>>>(a, e->bsum);
        k_scan_blocks<<<ny, 256, 0, st>>>(a, e->bsum);
        k_scan_apply<<<dim3(nt, ny), 256, 0, st>>>(a, e->bsum);
        HIPCHK(hipGetLastError());
        return PII_OK;
    }
    if (std::max(nb, nb2) > e->lb_cap) {
        const uint32_t cap = std::max(nb, nb2) + 64;
        int rc = grow(e, e->lb_state, 2 * (size_t)cap);
        if (rc) return rc;
        HIPCHK(hipMemsetAsync(e->lb_state, 0, 2 * (size_t)cap * 8, st));
        e->lb_cap = cap;
    }
    e->lb_epoch = (e->lb_epoch + 1) & 0xffffffu;
    if (e->lb_epoch == 0) e->lb_epoch = 1;
    // a pair of small scans (a re-scan step's lane and row scans) in one launch
    const LbArgs a{{in, in2 ? in2 : in}, {out, out2 ? out2 : out}, {n, n2}, {nb, nb2}, e->lb_cap};
    k_scan_lb<<<dim3(std::max(nb, nb2), in2 ? 2 : 1), LB_BLOCK, 0, st>>>(a, e->lb_state, e->lb_ticket, e->lb_epoch);
    HIPCHK(hipGetLastError());
    return PII_OK;
}

// scan lane size for a batch: 1 KiB lanes for big batches, down to 128 B so that a small batch (one
// re-scan step) still has ~64k lanes to spread over 256 CUs
uint32_t pick_lane_shift(const pii_engine* e, uint64_t total_bytes) {
    uint32_t sh = (uint32_t)__builtin_ctz(BYTES_PER_LANE);
    while (sh > MIN_LANE_SHIFT && (total_bytes >> sh) < (uint64_t)e->n_cu * 256) --sh;
    return sh;
}

// queues sized for a batch of `total_bytes`
int ensure_queues(pii_engine* e, uint64_t total_bytes) {
    int rc;
    if (e->pair_cap < total_bytes / 16 + 4096) {
        const uint64_t cap = total_bytes / 16 + 4096;
        if ((rc = grow_pairs(e, cap))) return rc;
        e->pair_cap = cap;
    }
    if (e->ev_cap < total_bytes / 16 + 4096) {
        const uint64_t cap = total_bytes / 16 + 4096;
        if ((rc = grow(e, e->evloc, cap))) return rc;
        e->ev_cap = cap;
    }
    return PII_OK;
}

// lanes of a batch of `total_bytes` whose base address is r0 mod 64 (slices are address aligned)
uint32_t lane_count(const pii_engine* e, uint64_t total_bytes) {
    if (total_bytes == 0) return 0;
    return (uint32_t)((total_bytes + e->r0 + (1u << e->lane_shift) - 1) >> e->lane_shift);
}

Geo make_geo(const pii_engine* e, const uint64_t* offs, uint32_t n_utt, uint32_t n_chunks, uint64_t base) {
    Geo g;
    g.offs = offs;
    g.first_utt = e->first_utt;
    g.lanes = e->lane_geo;
    g.base = base;
    g.n_utt = n_utt;
    g.n_chunks = n_chunks;
    g.sh = e->lane_shift;
    g.r0 = e->r0;
    g.long_min = e->long_min;
    return g;
}

// grid for the per-long-row kernels (they loop over the device-side row list)
uint32_t row_grid(const pii_engine* e, uint64_t total_bytes) {
    const uint64_t max_rows = total_bytes / 2048 + 1;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(max_rows, 2 * (uint64_t)e->n_cu));
}

// d_totals: 8 u64 totals, then the u64[max(T, 256)] per-infoType histogram
size_t hist_bytes(const pii_engine* e) { return 64 + (size_t)std::max(e->R.T, 256) * 8; }

// The stages every call shares: lane index, reverse DFA scan (+ the stitching of cut rows), (start,
// pattern) pair queue, context (segmented scan), leftmost-first confirmation.  Records tev[0..2].
int launch_front(pii_engine* e, const uint8_t* text, const uint64_t* offs, uint32_t n_utt, uint32_t n_chunks,
                 uint64_t base, uint64_t total_bytes, const uint32_t* slot, const uint8_t* role, const int64_t* ts,
                 int16_t* ctx, int16_t* win_ctx, const unsigned long long* pcount, hipStream_t st,
                 const uint32_t* err_init = nullptr, bool ctx_kernels = true, bool pair_first = true) {
    const RulesDev& R = e->R;
    e->epoch += 1;
    const Geo g = make_geo(e, offs, n_utt, n_chunks, base);
    // counter block (a second pass over the call starts from the first pass's), lane buckets, and the
    // histogram if pii_histogram_reset was called since the last call
    k_begin<<<1, 256, 0, st>>>(e->d_err, err_init, e->lane_bkt, n_chunks > 0 ? 2u * LANE_NB : 0u, e->hist,
                               e->hist_zero_pending ? (uint32_t)std::max(e->R.T, 256) : 0u);
    e->hist_zero_pending = false;
    if (e->timing >= 1) HIPCHK(hipEventRecord(e->tev[0], st));
    if (n_utt > 0) {
        k_chunk_index<<<(n_utt / CI_ROWS + 1 + 255) / 256, 256, 0, st>>>(offs, role, n_utt, n_chunks, e->lane_shift, e->r0,
                                                                e->long_min, R.kw_always_min, e->first_utt,
                                                                e->out_len, e->kw, win_ctx ? e->wc_n : nullptr,
                                                                e->long_rows, e->long_count, (uint32_t)e->cap_long, base,
                                                                total_bytes, e->d_err);
        if (e->long_min != NO_CUTS)
            k_fill_long<<<row_grid(e, total_bytes), 256, 0, st>>>(offs, n_utt, n_chunks, e->lane_shift, e->r0, e->long_rows,
                                                                   e->long_count, (uint32_t)e->cap_long, e->first_utt);
        if (n_chunks > 0) {
            // two chains per lane (k_scan2) for batches of full-size lanes; small batches (a re-scan
            // step: 128-512-byte lanes of one or two rows) have no utterance start to split at
            const bool split = e->scan2 && e->lane_shift == (uint32_t)__builtin_ctz(BYTES_PER_LANE) &&
                               e->long_min != NO_CUTS && e->n_sg == 1;
            const uint32_t nsb = (n_chunks + LANE_SORT_CHUNK - 1) / LANE_SORT_CHUNK;
            Geo g0 = g;
            g0.lanes = nullptr;
            (split ? k_lane_count<true> : k_lane_count<false>)<<<nsb, 256, 0, st>>>(g0, e->lane_bkt, e->lane_geo,
                                                                                    e->lane_spl);
            (split ? k_lane_place<true> : k_lane_place<false>)<<<nsb, 256, 0, st>>>(g, e->lane_bkt, e->lane_perm,
                                                                                    e->lane_pos, e->lane_spl);
            // one pass per SCAN group (one for the shipped rules): halo states, scan, stitching; the
            // utterance-start words are written once.  Several groups: group q on stream q mod
            // SCAN_STREAMS (forked after the words, joined before the pairs), so one pass's tail -- the
            // last workgroups of its longest-first lanes -- overlaps the next passes.
            const uint32_t ns_scan = e->n_sg > 1 ? 1 + e->n_aux : 1;
            const bool two = ns_scan > 1;
            for (uint32_t q = 0; q < e->n_sg; ++q) {
                const RulesDev& Rq = e->sg[q];
                Event* evq = e->ev + (uint64_t)q * e->cap_ev;
                uint32_t* cq = e->lane_cnt + (uint64_t)q * e->cap_lanes;
                uint32_t* stq = e->lane_st + 2ull * q * e->cap_lanes;
                if (q == 0 && split)
                    k_lane_bits2<<<(n_chunks + 255) / 256, 256, 0, st>>>(g, e->lane_pos, e->lane_spl,
                                                                         reinterpret_cast<uint32_t*>(e->bnd),
                                                                         e->lane_split);
                else if (q == 0)
                    k_lane_bits<<<(n_chunks + 255) / 256, 256, 0, st>>>(g, e->lane_pos, e->bnd);
                if (!SCAN_INLINE_HALO && e->long_min != NO_CUTS)
                    k_halo<<<row_grid(e, total_bytes), HALO_BLOCK, e->sg_lds[q], st>>>(Rq, g, text, e->long_rows,
                                                                                  e->long_count, stq, e->d_err);
                if (q == 0) {
                    if (e->timing >= 1) HIPCHK(hipEventRecord(e->kev[0], st));
                    if (two) {
                        HIPCHK(hipEventRecord(e->ev_fork, st));
                        for (uint32_t i = 0; i + 1 < ns_scan; ++i) HIPCHK(hipStreamWaitEvent(e->aux[i], e->ev_fork, 0));
                    }
                }
                const uint32_t si = q % ns_scan;
                const hipStream_t sq = si ? e->aux[si - 1] : st;
                // a WIDE table (row offsets / 2) that still leaves room for two workgroups per CU runs
                // at 768 threads too: 6 waves/SIMD instead of 4 (config 5: the 262 regex types' 70 KB
                // table); only the dictionary groups' ~100 KB tables need one 1024-thread workgroup
                const bool one_wg = e->sg_lds[q] > SCAN_LDS_TWO_WG;
                const int nt = one_wg ? SCAN_BLOCK_WIDE : SCAN_BLOCK;
                if (split) {
                    const int nt2 = one_wg ? SCAN_BLOCK_WIDE : SCAN2_BLOCK;
                    (q == 0 ? k_scan2<true> : one_wg ? k_scan2<false, SCAN_BLOCK_WIDE> : k_scan2<false>)<<<
                        (n_chunks + nt2 - 1) / nt2, nt2, e->sg_lds[q], sq>>>(
                        Rq, g, text, reinterpret_cast<const uint32_t*>(e->bnd), e->lane_split, e->lane_perm, evq,
                        cq, stq, e->d_err);
                } else {
                    const uint32_t nb = (n_chunks + nt - 1) / nt;
                    (q == 0 ? k_scan<true> : one_wg ? k_scan<false, SCAN_BLOCK_WIDE> : k_scan<false>)<<<
                        nb, nt, e->sg_lds[q], sq>>>(Rq, g, text, e->bnd, e->lane_perm, evq, cq, stq, e->d_err,
                                                    e->scan_ilv && nb <= e->n_cu ? nb : 0u);
                }
            }
            for (uint32_t i = 0; i + 1 < ns_scan; ++i) {
                HIPCHK(hipEventRecord(e->ev_join[i], e->aux[i]));
                HIPCHK(hipStreamWaitEvent(st, e->ev_join[i], 0));
            }
            if (e->timing >= 1) HIPCHK(hipEventRecord(e->kev[1], st));
            if (e->long_min != NO_CUTS)
                k_scan_fix<<<dim3(row_grid(e, total_bytes), e->n_sg), 256, e->max_sg_lds + FIX_LDS, st>>>(
                    e->d_sg, e->d_sg_lds, g, text, e->long_rows, e->long_count, e->ev, e->cap_ev, e->lane_cnt,
                    e->lane_st, e->cap_lanes, e->d_err);
            const uint32_t nbp = (n_chunks + PAIRS_BLOCK - 1) / PAIRS_BLOCK;
            const bool multi = e->n_sg > 1;
            const uint32_t ns = e->n_sg, cs = (uint32_t)e->cap_lanes;
            const uint64_t es = e->cap_ev;
            if (multi) HIPCHK(hipMemsetAsync(e->lane_np, 0, (size_t)n_chunks * sizeof(uint32_t), st));
            k_pairs_flat<false><<<dim3(nbp, ns), PAIRS_BLOCK, 0, st>>>(R, g, e->ev, e->lane_cnt, role, e->kw, e->evloc,
                                                                       e->pair_cap, e->ev_cap, e->lane_pair,
                                                                       e->lane_ev, e->lane_np, e->d_err, e->pres, e->acct,
                                                                       ns, es, cs, e->lane_evn);
            int rc;
            if ((rc = exclusive_scan(e, e->lane_np, n_chunks, e->lane_pair, st, multi ? e->lane_evn : e->lane_cnt,
                                     n_chunks, e->lane_ev)))
                return rc;
            // (no pair queue when no FIRST runs follow: the first pass of a full window re-scan and a
            // context-only call need the keyword groups of the count pass only, and cannot overflow it)
            if (!pair_first) {
            } else if (multi) {
                const uint32_t lpb = MERGE_WAVES * MERGE_LPW;
                k_pairs_merge<<<(n_chunks + lpb - 1) / lpb, MERGE_WAVES * 64, 0, st>>>(
                    g, e->ev, e->lane_cnt, e->evloc, e->pres, R.d_acc_off, R.d_acc_ids, e->pair_cap, e->ev_cap,
                    e->lane_pair, e->lane_ev, e->lane_np, e->d_err, ns, es, cs, e->acct, e->merge_cap);
            } else {
                k_pairs_flat<true><<<nbp, PAIRS_BLOCK, 0, st>>>(R, g, e->ev, e->lane_cnt, role, e->kw, e->evloc,
                                                                e->pair_cap, e->ev_cap, e->lane_pair,
                                                                e->lane_ev, e->lane_np, e->d_err, e->pres, e->acct,
                                                                1, 0, 0, nullptr);
            }
        }
        HIPCHK(hipGetLastError());
    }
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[1], st));
    const uint32_t nblk = (uint32_t)(((uint64_t)n_utt + CTX_TILE - 1) / CTX_TILE);
    if (n_utt > 0 && ctx_kernels) {
        // 16-byte row groups when the caller's arrays allow it
        const bool vec = ((uintptr_t)slot & 15) == 0 && ((uintptr_t)role & 7) == 0 && ((uintptr_t)ts & 15) == 0 &&
                         ((uintptr_t)ctx & 15) == 0 && ((uintptr_t)win_ctx & 15) == 0;
        (vec ? k_ctx_scan<true> : k_ctx_scan<false>)<<<nblk, CTX_THREADS, 0, st>>>(
            slot, role, e->kw, n_utt, e->n_slots, e->agg_v, e->agg_f, e->stamp, e->epoch, e->d_err);
        (vec ? k_ctx_apply<true> : k_ctx_apply<false>)<<<nblk, CTX_THREADS, 0, st>>>(
            slot, role, e->kw, ts, n_utt, e->n_slots, e->ttl_us, e->agg_v, e->agg_f, e->st_group, e->st_ts, ctx,
            e->commit, e->incl, e->ncommit, win_ctx);
        HIPCHK(hipGetLastError());
    }
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[2], st));
    if (n_utt > 0 && n_chunks > 0 && pair_first) {
        (e->img_first.global ? k_pair_first<true> : k_pair_first<false>)<<<e->n_seg, PAIR_BLOCK,
                                                                            e->img_first.global
                                                                                ? e->img_first_hot.li.total
                                                                                : e->img_first.lds(),
                                                                            st>>>(
            e->img_first.d, e->img_first.li, text, offs, pcount, e->pair_cap, e->evloc, e->pres, e->pend, e->matched,
            e->cont, e->mcount, e->d_err, e->img_first_hot.d, e->img_first_hot.li, e->first_p_hot);
        HIPCHK(hipGetLastError());
    }
    return PII_OK;
}

// The second pass of a full window re-scan (run_window_full): the joined windows as rows, each with the
// context group its window uses (no context kernels), the first pass's counter block, and the commits
// of the NEW rows (ring entries, context records) after a successful redaction.
struct WinFull {
    const int16_t* ctx_given;
    const uint32_t* err_init;
    WinRing W;
    WinBatch Bnew;
    const WNew* wnew;
    const uint32_t* slot_new;
    const int64_t* ts_new;
    const int32_t* kw_new;
    uint32_t n_new;
};

int run_pipeline(pii_engine* e, const uint8_t* text, const uint64_t* offs, uint32_t n_utt, uint64_t base,
                 uint64_t total_bytes, const uint32_t* slot, const uint8_t* role, const int64_t* ts, uint8_t* out,
                 uint64_t out_cap, uint64_t* out_offs, pii_span* spans, uint32_t span_cap, int16_t* ctx_info,
                 hipStream_t st, const pii_span* ext = nullptr, const uint32_t* ext_n = nullptr,
                 uint32_t ext_stride = 0, const WinFull* wf = nullptr) {
    if (total_bytes > PII_MAX_BATCH_BYTES || total_bytes + 2ull * n_utt + (total_bytes >> MIN_LANE_SHIFT) > 0xFFFFFFF0ull) {
        e->err = "batch larger than PII_MAX_BATCH_BYTES (positions and event arenas are 32-bit); split it";
        return PII_E_ARG;
    }
    const bool has_ext = ext != nullptr && n_utt > 0;
    if (has_ext && (!ext_n || ext_stride == 0)) {
        e->err = "external spans need their per-row counts and a stride > 0";
        return PII_E_ARG;
    }
    e->lane_shift = pick_lane_shift(e, total_bytes);
    e->r0 = (uint32_t)(((uintptr_t)text + base) & 63);
    e->long_min = 2u << e->lane_shift;          // rows longer than two lanes are cut
    const uint32_t n_chunks = lane_count(e, total_bytes);
    e->last_lanes = n_chunks;
    // external spans can be 1 byte long: the findings arenas are sized (and placed) for that
    RulesDev Rsel = e->R;
    if (has_ext) Rsel.min_len = 1;
    int rc = ensure_scratch(e, n_utt, total_bytes, n_chunks, Rsel.min_len);
    if (rc || (rc = ensure_queues(e, total_bytes)) || (rc = ensure_redact(e, span_cap, out_cap))) return rc;
    if (!wf) {                  // (a window call keeps its own record for pii_sync's re-run)
        e->last = pii_engine::Call{text, offs, n_utt, base, total_bytes, slot, role, ts, out, out_cap, out_offs, spans,
                                   span_cap, ctx_info, st, ext, ext_n, ext_stride};
        e->last_kind = 0;
    }
    const RulesDev& R = e->R;
    int16_t* ctx = wf ? const_cast<int16_t*>(wf->ctx_given) : ctx_info ? ctx_info : e->ctx;
    e->kev_valid = n_utt > 0 && total_bytes > 0;
    const Geo g = make_geo(e, offs, n_utt, n_chunks, base);
    // queue length = the lane-count scan's total (lane_pair[n_chunks]); 0 for an empty batch
    const unsigned long long* pcount =
        n_chunks > 0 ? reinterpret_cast<const unsigned long long*>(e->lane_pair + n_chunks) : e->pair_count;
    if ((rc = launch_front(e, text, offs, n_utt, n_chunks, base, total_bytes, slot, role, ts, ctx, nullptr, pcount,
                           st, wf ? wf->err_init : nullptr, wf == nullptr)))
        return rc;
    if (n_utt > 0 && n_chunks > 0) {
        if (e->img_eval_rg.d) {
            k_pair_eval<false, true><<<e->n_seg * e->eval_split, PAIR_BLOCK, e->img_eval_rg.lds(), st>>>(
                e->img_eval_rg.d, e->img_eval_rg.li, R.T, text, offs, role, ctx, pcount, e->pair_cap, e->matched,
                e->mcount, e->n_seg, e->evloc, e->pend, e->pres, reinterpret_cast<SelRec*>(e->cont), R.rule_off,
                R.rule_ids, e->eval_split);
        } else {
            (e->img_eval.global ? (e->lists_cl ? k_pair_eval<true, false, true> : k_pair_eval<true>)
                                : (e->lists_cl ? k_pair_eval<false, false, true> : k_pair_eval<false>))<<<
                e->n_seg * e->eval_split, PAIR_BLOCK,
                                                                             e->img_eval.lds(), st>>>(
                e->img_eval.d, e->img_eval.li, R.T, text, offs, role, ctx, pcount, e->pair_cap, e->matched,
                e->mcount, e->n_seg, e->evloc, e->pend, e->pres, reinterpret_cast<SelRec*>(e->cont), nullptr, nullptr,
                e->eval_split);
        }
        const bool xg = e->img_sel_rg.d != nullptr;
        const DevImage& isel = xg ? e->img_sel_rg : e->img_sel;
        const SelIO io{e->lane_pair, e->lane_np, reinterpret_cast<const SelRec*>(e->cont), e->pend, e->pair_cap, role, ctx, e->fd,
                       e->lane_nf, e->lane_rd, e->lane_reach, e->out_len, e->spill, ext, ext_n, ext_stride, e->d_err,
                       xg ? R.excl_off : nullptr, xg ? R.excl_ids : nullptr};
        const bool gi = isel.global;
        // (CL: the images hold deduplicated exclusion lists -- a large rule set; the RG path reads the
        // original tables from L2)
        const bool cl = e->lists_cl && !xg;
        auto ksel = cl ? (has_ext ? (gi ? k_select<true, true, true> : k_select<false, true, true>)
                                  : (gi ? k_select<true, false, true> : k_select<false, false, true>))
                       : (has_ext ? (gi ? k_select<true, true> : k_select<false, true>)
                                  : (gi ? k_select<true, false> : k_select<false, false>));
        auto kfix = cl ? (has_ext ? (gi ? k_sel_fix<true, true, true> : k_sel_fix<false, true, true>)
                                  : (gi ? k_sel_fix<true, false, true> : k_sel_fix<false, false, true>))
                       : (has_ext ? (gi ? k_sel_fix<true, true> : k_sel_fix<false, true>)
                                  : (gi ? k_sel_fix<true, false> : k_sel_fix<false, false>));
        ksel<<<(n_chunks + 255) / 256, 256, isel.lds(), st>>>(Rsel, isel.d, isel.li, g, io, e->d_err);
        const uint32_t rg = row_grid(e, total_bytes);
        k_sel_dirty<<<rg, ROW_BLOCK, 0, st>>>(g, e->long_rows, e->long_count, e->lane_reach, e->dirty, e->d_err);
        kfix<<<rg, 256, isel.lds(), st>>>(Rsel, isel.d, isel.li, g, io, e->long_rows, e->long_count,
                                                 e->dirty, e->d_err);
        k_rowlen<<<rg, ROW_BLOCK, 0, st>>>(g, e->long_rows, e->long_count, e->lane_rd, e->lane_rowbase, e->out_len,
                                          e->d_err);
        HIPCHK(hipGetLastError());
    }
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[3], st));
    // row output offsets and per-lane span offsets: one dual scan (a big batch: 3 launches instead of
    // 6; a small one: one single-pass look-back launch instead of 2)
    if (n_chunks > 0) {
        if ((rc = exclusive_scan(e, e->out_len, n_utt, out_offs, st, e->lane_nf, n_chunks, e->lane_sp))) return rc;
    } else {
        if ((rc = exclusive_scan(e, e->out_len, n_utt, out_offs, st))) return rc;
        if ((rc = exclusive_scan(e, e->lane_nf, n_chunks, e->lane_sp, st))) return rc;
    }
    k_finalize<<<1, 1, 0, st>>>(out_offs, e->lane_sp, n_utt, n_chunks, out_cap, span_cap, e->d_err, e->d_totals,
                                pcount, n_chunks > 0 ? e->lane_ev + n_chunks : nullptr, nullptr);
    HIPCHK(hipGetLastError());
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[4], st));
    if (n_utt > 0) {
        if (n_chunks > 0) {
            const uint32_t nsb = (n_chunks + 255) / 256;
            k_spans<<<nsb, 256, 0, st>>>(Rsel, g, e->fd, e->lane_nf, e->lane_sp, e->lane_rowbase, out_offs, e->d_err,
                                         spans, e->rsp, e->hist_part, e->hist_types);
            const uint32_t tiles = (uint32_t)((out_cap + 15) >> RTILE_SHIFT) + 1;
            k_tile_first<<<(tiles + 255) / 256, 256, 0, st>>>(R, e->rsp, e->lane_sp + n_chunks, out_offs + n_utt,
                                                              (uint32_t)((uintptr_t)out & 15), tiles, e->d_err,
                                                              e->tile_first);
            if (e->timing >= 1) HIPCHK(hipEventRecord(e->kev[2], st));
            k_redact<<<tiles, REDACT_BLOCK, 0, st>>>(R, text, offs, e->rsp, e->lane_sp + n_chunks, out_offs + n_utt,
                                                     total_bytes, e->tile_first, e->d_err, out);
            if (e->timing >= 1) HIPCHK(hipEventRecord(e->kev[3], st));
            if (!wf)        // (window findings are not counted, as on the incremental window path)
                k_hist_reduce<<<dim3(e->hist_types, std::max(1u, std::min(32u, nsb / 256))), 256, 0, st>>>(
                    e->hist_part, nsb, (int)e->hist_types, e->d_err, e->hist);
        }
        if (wf) {           // the new rows enter their rings; their context records are written
            k_win_commit<<<(uint32_t)(((uint64_t)wf->n_new * 16 + 255) / 256), 256, 0, st>>>(wf->W, wf->Bnew, wf->wnew,
                                                                                             e->d_err);
            k_ctx_commit<<<std::min<uint32_t>((wf->n_new + 255) / 256, 4 * e->n_cu), 256, 0, st>>>(
                wf->slot_new, wf->kw_new, wf->ts_new, e->incl, e->ncommit, e->commit, e->d_err, e->st_group, e->st_ts);
        } else {
            k_ctx_commit<<<std::min<uint32_t>((n_utt + 255) / 256, 4 * e->n_cu), 256, 0, st>>>(
                slot, e->kw, ts, e->incl, e->ncommit, e->commit, e->d_err, e->st_group, e->st_ts);
        }
        HIPCHK(hipGetLastError());
    }
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[5], st));
    HIPCHK(hipMemcpyAsync(e->h_totals, e->d_totals, hist_bytes(e), hipMemcpyDeviceToHost, st));
    e->h_hist_valid = true;
    HIPCHK(hipEventRecord(e->tev[6], st));
    return PII_OK;
}

int ensure_window_scratch(pii_engine* e, uint32_t n_utt) {
    int rc;
    if (e->wc_cap < e->pair_cap) {
        if ((rc = grow(e, e->wc, e->pair_cap)) || (rc = grow(e, e->phot, e->pair_cap))) return rc;
        e->wc_cap = e->pair_cap;
    }
    if (n_utt > e->wcap_utt) {
        const uint32_t nu = std::max<uint32_t>(n_utt + n_utt / 8, 1024);
        if ((rc = grow(e, e->wc_first, nu)) || (rc = grow(e, e->wc_n, nu)) || (rc = grow(e, e->wbound, nu)) ||
            (rc = grow(e, e->wfbase, (size_t)nu + 1)) || (rc = grow(e, e->n_wfind, nu)) ||
            (rc = grow(e, e->wout_len, nu)) || (rc = grow(e, e->wnew, nu)) || (rc = grow(e, e->wctx, nu)) ||
            (rc = grow(e, e->wspan_offs, (size_t)nu + 1)))
            return rc;
        e->wcap_utt = nu;
    }
    const uint64_t want = std::max<uint64_t>(4096, 4ull * n_utt);
    if (e->wfd_cap < want) {
        if ((rc = grow(e, e->wfd, want))) return rc;
        e->wfd_cap = want;
    }
    return PII_OK;
}

// the window history rings (pii_window_enable, pii_context_resize): persistent per-slot state, plain
// allocations outside the work-buffer accounting; empty rings
struct WinTables {
    WDesc* desc = nullptr;
    uint32_t *cnt = nullptr, *head = nullptr;
    uint8_t* arena = nullptr;
};
int alloc_window_tables(pii_engine* e, WinTables& w, size_t ns, uint32_t window_n, uint32_t slot_bytes) {
    const bool ok = hipMalloc(&w.desc, ns * window_n * sizeof(WDesc)) == hipSuccess &&
                    hipMalloc(&w.cnt, ns * 4) == hipSuccess && hipMalloc(&w.head, ns * 4) == hipSuccess &&
                    hipMalloc(&w.arena, ns * (size_t)slot_bytes) == hipSuccess &&
                    hipMemset(w.cnt, 0, ns * 4) == hipSuccess && hipMemset(w.head, 0, ns * 4) == hipSuccess;
    if (ok) return PII_OK;
    for (void* p : {(void*)w.desc, (void*)w.cnt, (void*)w.head, (void*)w.arena})
        if (p) (void)hipFree(p);
    w = WinTables{};
    (void)hipGetLastError();
    e->err = "device allocation failed: the window history rings";
    return PII_E_NOMEM;
}
void free_window_tables(pii_engine* e) {
    for (void* p : {(void*)e->wr_desc, (void*)e->wr_cnt, (void*)e->wr_head, (void*)e->wr_arena})
        if (p) (void)hipFree(p);
    e->wr_desc = nullptr;
    e->wr_cnt = e->wr_head = nullptr;
    e->wr_arena = nullptr;
}

int ensure_join(pii_engine* e, uint32_t n_utt) {
    int rc;
    if (n_utt + 1 > e->cap_j_utt) {
        const uint32_t nu = std::max<uint32_t>(n_utt + n_utt / 8 + 2, 1024);
        if ((rc = grow(e, e->jlen, nu)) || (rc = grow(e, e->joff, nu)) || (rc = grow(e, e->kw2, std::max(nu, e->cap_utt))) ||
            (rc = grow(e, e->jrole, nu)))
            return rc;
        HIPCHK(hipMemset(e->jrole, PII_ROLE_CUSTOMER, nu));
        e->cap_j_utt = nu;
    }
    if (!e->err_saved && (rc = grow(e, e->err_saved, 8))) return rc;
    if (!e->h_jtotal) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&e->h_jtotal), 8));
    return PII_OK;
}

// The full window re-scan (rule sets the incremental path cannot take, see k_win_jlen): pass 1 runs
// the shared front over the NEW rows for their keyword groups and the context every window uses
// (win_ctx), plans the ring commits (text only) and measures the joined windows; one host wait reads
// the joined size; the windows are materialised; pass 2 is the ordinary pipeline over them as
// CUSTOMER rows with the given context groups, then the new rows enter their rings and the context
// records are written -- only when every stage succeeded.
int run_window_full(pii_engine* e, const uint8_t* text, const uint64_t* offs, uint32_t n_utt, uint64_t base,
                    uint64_t total_bytes, const uint32_t* slot, const uint8_t* role, const int64_t* ts, uint8_t* out,
                    uint64_t out_cap, uint64_t* out_offs, pii_span* spans, uint32_t span_cap, int16_t* win_ctx,
                    hipStream_t st) {
    e->lane_shift = pick_lane_shift(e, total_bytes);
    e->r0 = (uint32_t)(((uintptr_t)text + base) & 63);
    e->long_min = 2u << e->lane_shift;
    const uint32_t n_chunks = lane_count(e, total_bytes);
    e->last_lanes = n_chunks;
    int rc = ensure_scratch(e, n_utt, total_bytes, n_chunks);
    if (rc || (rc = ensure_queues(e, total_bytes)) || (rc = ensure_window_scratch(e, n_utt)) || (rc = ensure_join(e, n_utt)))
        return rc;
    e->last = pii_engine::Call{text, offs, n_utt, base, total_bytes, slot, role, ts, out, out_cap, out_offs, spans,
                               span_cap, win_ctx, st, nullptr, nullptr, 0};
    e->last_kind = 1;
    int16_t* wctx = win_ctx ? win_ctx : e->wctx;
    const unsigned long long* pcount =
        n_chunks > 0 ? reinterpret_cast<const unsigned long long*>(e->lane_pair + n_chunks) : e->pair_count;
    if ((rc = launch_front(e, text, offs, n_utt, n_chunks, base, total_bytes, slot, role, ts, e->ctx, wctx, pcount, st,
                           nullptr, true, false)))
        return rc;
    const WinRing W{e->wr_desc, e->wr_cnt, e->wr_head, e->wr_arena, e->win_n, e->win_slot_bytes, e->n_slots, 0};
    if (n_utt) HIPCHK(hipMemsetAsync(e->wc_n, 0, (size_t)n_utt * 4, st));      // text-only ring entries
    const WinBatch B{text, offs, slot, e->wc, e->wc_first, e->wc_n, n_utt};
    const uint32_t nb = (n_utt + 255) / 256;
    if (n_utt) {
        k_win_plan<<<nb, 256, 0, st>>>(W, B, e->wbound, e->wnew, e->d_err);
        k_win_alloc<<<nb, 256, 0, st>>>(W, B, e->wnew, e->d_err);
        k_win_jlen<<<nb, 256, 0, st>>>(W, B, e->jlen, e->d_err);
    }
    k_err_save<<<1, 1, 0, st>>>(e->d_err, e->err_saved);
    HIPCHK(hipGetLastError());
    if ((rc = exclusive_scan(e, e->jlen, n_utt, e->joff, st))) return rc;
    HIPCHK(hipMemcpyAsync(e->h_jtotal, e->joff + n_utt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t jt = *e->h_jtotal;
    if (jt > PII_MAX_BATCH_BYTES || jt + 2ull * n_utt + (jt >> MIN_LANE_SHIFT) > 0xFFFFFFF0ull) {
        e->err = "the call's joined windows exceed PII_MAX_BATCH_BYTES; split the batch";
        return PII_E_ARG;
    }
    if (jt + 64 > e->cap_jbuf) {
        if ((rc = grow(e, e->jbuf, jt + jt / 8 + 64))) return rc;
        e->cap_jbuf = jt + jt / 8 + 64;
    }
    if (n_utt) k_win_join<<<(n_utt + 3) / 4, 256, 0, st>>>(W, B, e->joff, e->jbuf, e->d_err);
    HIPCHK(hipGetLastError());
    int32_t* kwA = e->kw;                // pass 2 must not overwrite the new rows' keyword groups
    e->kw = e->kw2;
    const WinFull wf{wctx, e->err_saved, W, B, e->wnew, slot, ts, kwA, n_utt};
    rc = run_pipeline(e, e->jbuf, e->joff, n_utt, 0, jt, slot, e->jrole, ts, out, out_cap, out_offs, spans, span_cap,
                      nullptr, st, nullptr, nullptr, 0, &wf);
    e->kw = kwA;
    return rc;
}

// the window re-scan call (a12): the shared front over the NEW rows only, then resident candidates,
// window selection, window redaction, ring commit
int run_window(pii_engine* e, const uint8_t* text, const uint64_t* offs, uint32_t n_utt, uint64_t base,
               uint64_t total_bytes, const uint32_t* slot, const uint8_t* role, const int64_t* ts, uint8_t* out, uint64_t out_cap,
               uint64_t* out_offs, pii_span* spans, uint32_t span_cap, int16_t* win_ctx, hipStream_t st) {
    if (e->win_n == 0) {
        e->err = "window re-scan not enabled (pii_window_enable)";
        return PII_E_ARG;
    }
    if (total_bytes > PII_MAX_BATCH_BYTES || total_bytes + 2ull * n_utt + (total_bytes >> MIN_LANE_SHIFT) > 0xFFFFFFF0ull) {
        e->err = "batch larger than PII_MAX_BATCH_BYTES (positions and event arenas are 32-bit); split it";
        return PII_E_ARG;
    }
    if (e->win_full)
        return run_window_full(e, text, offs, n_utt, base, total_bytes, slot, role, ts, out, out_cap, out_offs, spans,
                               span_cap, win_ctx, st);
    e->lane_shift = pick_lane_shift(e, total_bytes);
    e->r0 = (uint32_t)(((uintptr_t)text + base) & 63);
    // rows whole by default; PII_WIN_LONG = n cuts rows longer than n lanes like the main path's long
    // rows (k_win_cands then walks a cut row whole).  A step's scan takes as long as its longest lane
    // (a whole 750-byte row of 128-byte lanes), and cutting at 2 lanes takes k_scan 67 -> 53 us, but
    // the stitching, the long-row list and the cut-row candidate walk cost more
    e->long_min = e->win_long ? e->win_long << e->lane_shift : NO_CUTS;
    const uint32_t n_chunks = lane_count(e, total_bytes);
    e->last_lanes = n_chunks;
    int rc = ensure_scratch(e, n_utt, total_bytes, n_chunks);
    if (rc || (rc = ensure_queues(e, total_bytes)) || (rc = ensure_window_scratch(e, n_utt))) return rc;
    e->last = pii_engine::Call{text, offs, n_utt, base, total_bytes, slot, role, ts, out, out_cap, out_offs, spans,
                               span_cap, win_ctx, st};
    e->last_kind = 1;
    const RulesDev& R = e->R;
    int16_t* wctx = win_ctx ? win_ctx : e->wctx;
    e->kev_valid = n_utt > 0 && total_bytes > 0;
    const unsigned long long* pcount =
        n_chunks > 0 ? reinterpret_cast<const unsigned long long*>(e->lane_pair + n_chunks) : e->pair_count;
    if ((rc = launch_front(e, text, offs, n_utt, n_chunks, base, total_bytes, slot, role, ts, e->ctx, wctx, pcount,
                           st)))
        return rc;
    if (n_utt > 0 && n_chunks > 0) {
        (e->img_eval.global ? k_win_eval<true> : k_win_eval<false>)<<<e->n_seg, PAIR_BLOCK, e->img_eval.lds(), st>>>(
            e->img_eval.d, e->img_eval.li, text, offs, pcount, e->pair_cap, e->matched, e->mcount, e->n_seg,
            e->evloc, e->pend, e->pres, e->phot);
        k_win_cands<<<(n_chunks + 255) / 256, 256, 0, st>>>(make_geo(e, offs, n_utt, n_chunks, base), e->lane_pair, e->lane_np, e->evloc, e->pres,
                                                            e->pend, e->phot, e->pair_cap, e->spill, e->wc, e->wc_first,
                                                            e->wc_n, e->d_err);
        HIPCHK(hipGetLastError());
    }
    const WinRing W{e->wr_desc, e->wr_cnt, e->wr_head, e->wr_arena, e->win_n, e->win_slot_bytes, e->n_slots, 0};
    const WinBatch B{text, offs, slot, e->wc, e->wc_first, e->wc_n, n_utt};
    const uint32_t nb = (n_utt + 255) / 256;
    if (n_utt > 0 && n_chunks > 0 && R.n_hot > 0) {
        // (the image in LDS when it fits beside the halo tables, else read in place)
        const bool hg = e->img_eval.global || ((size_t)e->img_eval.li.total + 15) / 16 * 16 + HALO_LDS > IMG_LDS_MAX;
        const size_t hl = (hg ? 0 : ((size_t)e->img_eval.li.total + 15) / 16 * 16) + HALO_LDS;
        (hg ? k_win_halo<true> : k_win_halo<false>)<<<(n_utt + HALO_ROWS - 1) / HALO_ROWS, HALO_ROWS, hl, st>>>(
            e->img_eval.d, e->img_eval.li, W, B, e->wc, e->halo_items, e->d_err);
    }
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[3], st));
    if (n_utt > 0) {
        k_win_plan<<<nb, 256, 0, st>>>(W, B, e->wbound, e->wnew, e->d_err);
        if ((rc = exclusive_scan(e, e->wbound, n_utt, e->wfbase, st))) return rc;
        (e->img_wsel.global ? k_win_select<true> : k_win_select<false>)<<<nb, 256, e->img_wsel.lds(), st>>>(
            R, e->img_wsel.d, e->img_wsel.li, W, B, wctx, e->wfbase,
                                                             e->wfd_cap, e->wfd, e->n_wfind, e->wout_len, e->d_err);
        HIPCHK(hipGetLastError());
    }
    if (n_utt > 0) {
        if ((rc = exclusive_scan(e, e->wout_len, n_utt, out_offs, st, e->n_wfind, n_utt, e->wspan_offs))) return rc;
    } else {
        if ((rc = exclusive_scan(e, e->wout_len, n_utt, out_offs, st))) return rc;
        if ((rc = exclusive_scan(e, e->n_wfind, n_utt, e->wspan_offs, st))) return rc;
    }
    if (n_utt > 0) k_win_alloc<<<nb, 256, 0, st>>>(W, B, e->wnew, e->d_err);
    k_finalize<<<1, 1, 0, st>>>(out_offs, e->wspan_offs, n_utt, n_utt, out_cap, span_cap, e->d_err, e->d_totals,
                                pcount, n_chunks > 0 ? e->lane_ev + n_chunks : nullptr, n_utt > 0 ? e->wfbase + n_utt : nullptr);
    HIPCHK(hipGetLastError());
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[4], st));
    if (n_utt > 0) {
        if (e->timing >= 1) HIPCHK(hipEventRecord(e->kev[2], st));
        k_win_redact<<<(n_utt + WIN_TILE - 1) / WIN_TILE, REDACT_BLOCK, 0, st>>>(
            R, W, B, e->wfd, e->wfbase, e->n_wfind, out_offs, e->wspan_offs, e->d_err, out, spans);
        if (e->timing >= 1) HIPCHK(hipEventRecord(e->kev[3], st));
        k_win_commit<<<(uint32_t)(((uint64_t)n_utt * 16 + 255) / 256), 256, 0, st>>>(W, B, e->wnew, e->d_err);
        k_ctx_commit<<<std::min<uint32_t>(nb, 4 * e->n_cu), 256, 0, st>>>(slot, e->kw, ts, e->incl, e->ncommit,
                                                                          e->commit, e->d_err, e->st_group, e->st_ts);
        HIPCHK(hipGetLastError());
    }
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[5], st));
    HIPCHK(hipMemcpyAsync(e->h_totals, e->d_totals, hist_bytes(e), hipMemcpyDeviceToHost, st));
    e->h_hist_valid = true;
    HIPCHK(hipEventRecord(e->tev[6], st));
    return PII_OK;
}

// pii_context_update: the shared front without the pair queue or FIRST runs (the count pass yields the
// AGENT rows' keyword groups), the context kernels and the context commit
int run_context(pii_engine* e, const uint8_t* text, const uint64_t* offs, uint32_t n_utt, uint64_t total_bytes,
                const uint32_t* slot, const uint8_t* role, const int64_t* ts, int16_t* ctx_info, hipStream_t st) {
    if (total_bytes > PII_MAX_BATCH_BYTES || total_bytes + 2ull * n_utt + (total_bytes >> MIN_LANE_SHIFT) > 0xFFFFFFF0ull) {
        e->err = "batch larger than PII_MAX_BATCH_BYTES (positions and event arenas are 32-bit); split it";
        return PII_E_ARG;
    }
    e->lane_shift = pick_lane_shift(e, total_bytes);
    e->r0 = (uint32_t)((uintptr_t)text & 63);
    e->long_min = 2u << e->lane_shift;
    const uint32_t n_chunks = lane_count(e, total_bytes);
    e->last_lanes = n_chunks;
    int rc = ensure_scratch(e, n_utt, total_bytes, n_chunks);
    if (rc) return rc;
    e->last = pii_engine::Call{text, offs, n_utt, 0, total_bytes, slot, role, ts, nullptr, 0, nullptr, nullptr,
                               0, ctx_info, st, nullptr, nullptr, 0};
    e->last_kind = 2;
    e->kev_valid = false;
    const unsigned long long* pcount =
        n_chunks > 0 ? reinterpret_cast<const unsigned long long*>(e->lane_pair + n_chunks) : e->pair_count;
    if ((rc = launch_front(e, text, offs, n_utt, n_chunks, 0, total_bytes, slot, role, ts, ctx_info, nullptr, pcount,
                           st, nullptr, true, false)))
        return rc;
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[3], st));
    k_ctx_totals<<<1, 1, 0, st>>>(e->d_err, e->d_totals);
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[4], st));
    if (n_utt > 0)
        k_ctx_commit<<<std::min<uint32_t>((n_utt + 255) / 256, 4 * e->n_cu), 256, 0, st>>>(
            slot, e->kw, ts, e->incl, e->ncommit, e->commit, e->d_err, e->st_group, e->st_ts);
    HIPCHK(hipGetLastError());
    if (e->timing >= 2) HIPCHK(hipEventRecord(e->tev[5], st));
    HIPCHK(hipMemcpyAsync(e->h_totals, e->d_totals, 64, hipMemcpyDeviceToHost, st));
    e->h_hist_valid = false;
    HIPCHK(hipEventRecord(e->tev[6], st));
    return PII_OK;
}

int rerun_last(pii_engine* e) {
    const pii_engine::Call c = e->last;
    if (e->last_kind == 2)
        return run_context(e, c.text, c.offs, c.n_utt, c.total, c.slot, c.role, c.ts, c.ctx_info, c.st);
    if (e->last_kind == 1)
        return run_window(e, c.text, c.offs, c.n_utt, c.base, c.total, c.slot, c.role, c.ts, c.out, c.out_cap,
                          c.out_offs, c.spans, c.span_cap, c.ctx_info, c.st);
    return run_pipeline(e, c.text, c.offs, c.n_utt, c.base, c.total, c.slot, c.role, c.ts, c.out, c.out_cap,
                        c.out_offs, c.spans, c.span_cap, c.ctx_info, c.st, c.ext, c.ext_n, c.ext_stride);
}

struct ExtArgs {
    const pii_span* ext;
    const uint32_t* ext_n;
    uint32_t stride;
};
int device_call(pii_engine* e, bool window, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                const uint32_t* d_slot, const uint8_t* d_role, const int64_t* d_ts, uint8_t* d_out, uint64_t out_cap,
                uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap, int16_t* d_ctx_info, void* stream,
                const uint64_t* declared, const ExtArgs* x = nullptr);
}  // namespace

extern "C" {

const char* pii_last_error(pii_engine* e) { return e ? e->err.c_str() : "null engine"; }

int pii_engine_create(const void* blob, size_t n, int device, uint32_t n_conv_slots, int64_t ttl_us,
                      pii_engine** out) {
    if (!blob || !out) return PII_E_ARG;
    *out = nullptr;
    std::vector<Section> secs;
    if (!parse_blob(static_cast<const uint8_t*>(blob), n, secs)) return PII_E_RULES;
    auto find = [&](const char* nm) -> const Section* {
        for (auto& s : secs)
            if (s.name == nm) return &s;
        return nullptr;
    };
    static const char* req[] = {"meta", "scan.cmap2", "scan.d.trans", "scan.d.accid", "scan.d.acc_off",
                                "scan.d.acc_ids", "scan.k.trans", "scan.k.accid", "scan.k.acc_off", "scan.k.acc_ids",
                                "det.type", "det.validator", "det.lik", "det.exidx", "det.first_desc", "hot.rule",
                                "hot.dfa_desc", "pool.trans", "pool.flags", "pool.cmap", "var.enabled",
                                "var.minlik", "var.rule_off", "var.rule_ids", "var.excl_off", "var.excl_ids",
                                "kw.type", "kw.always", "types.names"};
    for (auto r : req)
        if (!find(r)) return PII_E_RULES;
    const int64_t* meta = reinterpret_cast<const int64_t*>(find("meta")->data);
    pii_engine* e = new pii_engine();
    e->device = device;
    e->n_slots = n_conv_slots;
    e->ttl_us = ttl_us;
    RulesDev& R = e->R;
    R.P = (int)meta[0];
    R.G = (int)meta[1];
    R.T = (int)meta[2];
    R.V = (int)meta[3];
    R.SD = (int)meta[4];
    R.CD = (int)meta[5];
    R.d_start = (int)meta[6];
    R.SK = (int)meta[7];
    R.CK = (int)meta[8];
    R.k_start = (int)meta[9];
    R.n_hot = (int)meta[10];
    R.min_len = (int)std::max<int64_t>(1, meta[11]);
    e->window_ok = meta[13] != 0;
    auto fail = [&](const char* why) {
        e->err = why;
        pii_engine_destroy(e);
        return PII_E_RULES;
    };
    if (R.P > 65535) return fail("too many detector patterns");
    // scan table entries are 16-bit LDS byte addresses (k_scan layout: class map, D rows, K rows);
    // rows are padded to an even class count so every row address is a multiple of 4 and bit 1 of
    // an entry is free for the destination's end-of-text accept
    R.CDs = (R.CD + 1) & ~1;
    R.CKs = (R.CK + 1) & ~1;
    R.dsh = 0;
    const uint32_t td_words = (uint32_t)(R.SD * R.CDs / 2), tk_words = (uint32_t)(R.SK * R.CKs / 2);
    const uint32_t tk_base = SCAN_TD_BASE + td_words * 4;
    if ((uint64_t)tk_base + (uint64_t)tk_words * 4 > 65536) return fail("SCAN tables exceed 64 KiB of LDS");
    if (R.T > 65535) return fail("too many types");
    // names + tokens
    {
        const Section* s = find("types.names");
        const char* p = reinterpret_cast<const char*>(s->data);
        size_t i = 0;
        while (i < s->bytes) {
            size_t l = strnlen(p + i, s->bytes - i);
            e->names.emplace_back(p + i, l);
            i += l + 1;
        }
        if ((int)e->names.size() != R.T) return fail("type table mismatch");
    }
    {
        const Section* s = find("kw.type");
        const uint16_t* k = reinterpret_cast<const uint16_t*>(s->data);
        for (int g = 0; g < R.G; ++g) e->kw_type.push_back(k[g]);
    }
    // host-side derived tables
    std::vector<uint16_t> td(R.SD * R.CDs, 0), tk(R.SK * R.CKs, 0), dacc(R.SD * R.CDs, 0), kacc(R.SK * R.CKs, 0);
    // entry (row, class) = address of the destination row | accept | accept of the destination's
    // end-of-text transition (class C-1) << 1, so k_scan resets at an utterance start without
    // reading the end-of-text entry
    // (k_scan: rows are placed with the START state first -- row = pos(state) -- and entries are the
    // destination row's byte offset from the table base, so a reset is "row 0"; the class words carry
    // the table bases; accept-id tables follow the same placement)
    auto relayout = [](const uint16_t* s, const uint16_t* acc, int S, int C, int Cs, int start, uint16_t* t,
                       uint16_t* a, int dsh = 0) {
        auto pos = [start](uint32_t r) { return r == (uint32_t)start ? 0u : r == 0 ? (uint32_t)start : r; };
        for (int r = 0; r < S; ++r)
            for (int c = 0; c < C; ++c) {
                const uint32_t v = s[r * C + c], dst = v & 0x7fff;
                const uint32_t eot = s[dst * C + C - 1] >> 15;
                t[pos(r) * Cs + c] = (uint16_t)(((pos(dst) * Cs * 2) >> dsh) | (v >> 15) | (eot << 1));
                a[pos(r) * Cs + c] = acc[r * C + c];
            }
    };
    {
        relayout(reinterpret_cast<const uint16_t*>(find("scan.d.trans")->data),
                 reinterpret_cast<const uint16_t*>(find("scan.d.accid")->data), R.SD, R.CD, R.CDs, R.d_start,
                 td.data(), dacc.data());
        relayout(reinterpret_cast<const uint16_t*>(find("scan.k.trans")->data),
                 reinterpret_cast<const uint16_t*>(find("scan.k.accid")->data), R.SK, R.CK, R.CKs, R.k_start,
                 tk.data(), kacc.data());
    }
    R.d_start = R.k_start = 0;                                     // row offsets: the start rows are first
    std::vector<uint32_t> cmap4(256);
    {
        const uint16_t* c2 = reinterpret_cast<const uint16_t*>(find("scan.cmap2")->data);
        for (int b = 0; b < 256; ++b)
            cmap4[b] = (SCAN_TD_BASE + 2u * (c2[b] & 0xffu)) | (tk_base + 2u * (uint32_t)(c2[b] >> 8)) << 16;
    }
    std::vector<uint16_t> k_acc_min;
    {
        const Section* so = find("scan.k.acc_off");
        const uint32_t* off = reinterpret_cast<const uint32_t*>(so->data);
        const uint16_t* ids = reinterpret_cast<const uint16_t*>(find("scan.k.acc_ids")->data);
        const size_t nsets = so->bytes / 4 - 1;
        R.n_kacc = (uint32_t)nsets;
        R.n_dacc = (uint32_t)(find("scan.d.acc_off")->bytes / 4 - 1);
        for (size_t a = 0; a < nsets; ++a) {
            int m = KW_NONE;
            for (uint32_t i = off[a]; i < off[a + 1]; ++i) m = std::min<int>(m, ids[i]);
            k_acc_min.push_back((uint16_t)m);
        }
    }
    R.kw_always_min = KW_NONE;
    {
        const uint8_t* al = find("kw.always")->data;
        for (int g = 0; g < R.G; ++g)
            if (al[g]) {
                R.kw_always_min = g;
                break;
            }
    }
    {
        const uint8_t* ex = find("det.exidx")->data;
        int ne = 0;
        for (int p = 0; p < R.P; ++p)
            if (ex[p] != 0xff) ne = std::max(ne, ex[p] + 1);
        if (ne > NE_MAX) return fail("too many excluder patterns");
        R.NE = ne;
    }
    std::vector<uint32_t> tok_off(R.T + 1, 0);
    std::string tok;
    for (int t = 0; t < R.T; ++t) {
        tok += "[" + e->names[t] + "]";
        tok_off[t + 1] = (uint32_t)tok.size();
    }
    tok += "\n";               // the re-scan window separator (k_win_redact piece source)
    R.nl_off = (uint32_t)tok.size() - 1;
    tok.append(32, '\0');     // k_redact reads aligned 16-byte windows past a token's end
    // SCAN groups >= 1: their own D automaton and class map, a 1-row never-accepting K stub
    struct HostGroup {
        int SD, CD, CDs, start, dsh;
        uint32_t lds;
        std::vector<uint16_t> td, tk, dacc, kacc, npair;
        std::vector<uint32_t> cmap4;
    };
    std::vector<HostGroup> hg;
    {
        const int64_t n_extra = meta[14];
        if (n_extra < 0 || n_extra + 1 > SCAN_GROUPS_MAX) return fail("too many SCAN groups");
        const Section* gs = find("scan.groups");
        if (n_extra > 0 && (!gs || gs->bytes < (size_t)n_extra * 32)) return fail("SCAN group table missing");
        for (int64_t q = 1; q <= n_extra; ++q) {
            const int64_t* gm = reinterpret_cast<const int64_t*>(gs->data) + 4 * (q - 1);
            const std::string nm = "scan.g" + std::to_string(q);
            const Section *sc = find((nm + ".cmap").c_str()), *st = find((nm + ".trans").c_str()),
                          *sa = find((nm + ".accid").c_str());
            HostGroup h;
            h.SD = (int)gm[0];
            h.CD = (int)gm[1];
            h.CDs = (h.CD + 1) & ~1;
            h.dsh = 0;
            if (!sc || !st || !sa || st->bytes != (size_t)h.SD * h.CD * 2 || sa->bytes != st->bytes || sc->bytes != 256)
                return fail("SCAN group tables malformed");
            // a table past 64 KiB of LDS addresses is WIDE: rows padded to a multiple of 4 entries (8-byte
            // aligned), entries hold the row offset / 2, so 16-bit entries reach 128 KiB (and the u16
            // transition index of an event, 64k entries)
            if (SCAN_TD_BASE + (size_t)h.SD * h.CDs * 2 + 4 + SCAN_SPREAD_BYTES > 65536) {
                h.CDs = (h.CD + 3) & ~3;
                h.dsh = 1;
                if ((size_t)h.SD * h.CDs > 65536) return fail("a SCAN group exceeds 128 KiB of LDS");
            }
            const uint32_t tkb = SCAN_TD_BASE + (uint32_t)(h.SD * h.CDs) * 2;
            h.lds = tkb + 4 + SCAN_SPREAD_BYTES;                // + the K stub's row (2 entries), spread masks
            if (h.lds + FIX_LDS > 160 * 1024) return fail("a SCAN group exceeds the LDS");
            h.td.assign((size_t)h.SD * h.CDs, 0);
            h.dacc.assign((size_t)h.SD * h.CDs, 0);
            if (gm[2] < 0 || gm[2] >= h.SD) return fail("SCAN group start state out of range");
            relayout(reinterpret_cast<const uint16_t*>(st->data), reinterpret_cast<const uint16_t*>(sa->data), h.SD,
                     h.CD, h.CDs, (int)gm[2], h.td.data(), h.dacc.data(), h.dsh);
            h.tk = {0, 0};
            h.kacc = {0, 0};
            h.start = 0;
            h.cmap4.resize(256);
            // class words of a group >= 1: the D half only (its K is the stub, stepped at tk_base)
            for (int b = 0; b < 256; ++b) h.cmap4[b] = SCAN_TD_BASE + 2u * sc->data[b];
            hg.push_back(std::move(h));
        }
    }
    // one device buffer holding every table, 256-byte aligned sections
    struct Put {
        const void* src;
        size_t bytes;
        size_t off;
    };
    std::vector<Put> puts;
    size_t total = 0;
    auto add = [&](const void* src, size_t bytes) {
        total = (total + 255) & ~(size_t)255;
        puts.push_back({src, bytes, total});
        total += bytes + 16;
        return puts.size() - 1;
    };
    auto addsec = [&](const char* nm) { return add(find(nm)->data, find(nm)->bytes); };
    size_t i_cmap = add(cmap4.data(), cmap4.size() * 4), i_td = add(td.data(), td.size() * 2), i_tk = add(tk.data(), tk.size() * 2);
    size_t i_dacc = add(dacc.data(), dacc.size() * 2), i_doff = addsec("scan.d.acc_off"), i_dids = addsec("scan.d.acc_ids");
    size_t i_kacc = add(kacc.data(), kacc.size() * 2), i_kmin = add(k_acc_min.data(), k_acc_min.size() * 2);
    std::vector<uint16_t> d_npair(dacc.size()), k_grp(kacc.size());
    {
        const uint32_t* off = reinterpret_cast<const uint32_t*>(find("scan.d.acc_off")->data);
        for (size_t i = 0; i < dacc.size(); ++i) d_npair[i] = (uint16_t)(off[dacc[i] + 1] - off[dacc[i]]);
        for (size_t i = 0; i < kacc.size(); ++i) k_grp[i] = kacc[i] ? k_acc_min[kacc[i]] : (uint16_t)KW_NONE;
        for (auto& h : hg) {
            h.npair.resize(h.dacc.size());
            for (size_t i = 0; i < h.dacc.size(); ++i) h.npair[i] = (uint16_t)(off[h.dacc[i] + 1] - off[h.dacc[i]]);
        }
    }
    size_t i_dnp = add(d_npair.data(), d_npair.size() * 2), i_kgrp = add(k_grp.data(), k_grp.size() * 2);
    size_t i_dt = addsec("det.type"), i_dv = addsec("det.validator"), i_dl = addsec("det.lik"),
           i_dx = addsec("det.exidx"), i_fd = addsec("det.first_desc"), i_hr = addsec("hot.rule"),
           i_hd = addsec("hot.dfa_desc"), i_ve = addsec("var.enabled"), i_vm = addsec("var.minlik"),
           i_ro = addsec("var.rule_off"), i_ri = addsec("var.rule_ids"), i_eo = addsec("var.excl_off"),
           i_ei = addsec("var.excl_ids"), i_to = add(tok_off.data(), tok_off.size() * 4),
           i_tb = add(tok.data(), tok.size());
    struct GroupPut { size_t cmap, td, tk, dacc, kacc, npair; };
    std::vector<GroupPut> gp;
    for (auto& h : hg)
        gp.push_back({add(h.cmap4.data(), 1024), add(h.td.data(), h.td.size() * 2), add(h.tk.data(), 4),
                      add(h.dacc.data(), h.dacc.size() * 2), add(h.kacc.data(), 4),
                      add(h.npair.data(), h.npair.size() * 2)});
    if (hipSetDevice(device) != hipSuccess) { e->err = "hipSetDevice failed"; pii_engine_destroy(e); return PII_E_DEVICE; }
    if (hipMalloc(&e->d_rules, total) != hipSuccess) return fail("hipMalloc rules failed");
    std::vector<uint8_t> host(total, 0);
    for (auto& p : puts) std::memcpy(host.data() + p.off, p.src, p.bytes);
    if (hipMemcpy(e->d_rules, host.data(), total, hipMemcpyHostToDevice) != hipSuccess) return fail("upload failed");
    uint8_t* b = static_cast<uint8_t*>(e->d_rules);
    auto at = [&](size_t i) { return b + puts[i].off; };
    R.cmap4 = (const uint32_t*)at(i_cmap);
    R.td = (const uint16_t*)at(i_td);
    R.tk = (const uint16_t*)at(i_tk);
    R.d_accid = (const uint16_t*)at(i_dacc);
    R.d_acc_off = (const uint32_t*)at(i_doff);
    R.d_acc_ids = (const uint16_t*)at(i_dids);
    R.k_accid = (const uint16_t*)at(i_kacc);
    R.k_acc_min = (const uint16_t*)at(i_kmin);
    R.d_npair = (const uint16_t*)at(i_dnp);
    R.k_grp = (const uint16_t*)at(i_kgrp);
    R.det_type = (const uint16_t*)at(i_dt);
    R.det_val = (const uint8_t*)at(i_dv);
    R.det_lik = (const uint8_t*)at(i_dl);
    R.det_exidx = (const uint8_t*)at(i_dx);
    R.first_desc = (const int32_t*)at(i_fd);
    R.hot_rule = (const int32_t*)at(i_hr);
    R.hot_desc = (const int32_t*)at(i_hd);
    R.var_enabled = (const uint8_t*)at(i_ve);
    R.var_minlik = (const uint8_t*)at(i_vm);
    R.rule_off = (const uint32_t*)at(i_ro);
    R.rule_ids = (const uint16_t*)at(i_ri);
    R.excl_off = (const uint32_t*)at(i_eo);
    R.excl_ids = (const uint16_t*)at(i_ei);
    R.tok_off = (const uint32_t*)at(i_to);
    R.tok_bytes = (const uint8_t*)at(i_tb);
    if (R.n_dacc >= 65535) return fail("too many SCAN accept sets");
    {   // per-kernel LDS images
        auto sec = [&](const char* nm) { return std::make_pair((const void*)find(nm)->data, (size_t)find(nm)->bytes); };
        const uint16_t* ptrans = (const uint16_t*)find("pool.trans")->data;
        const uint8_t* pflags = (const uint8_t*)find("pool.flags")->data;
        const uint8_t* pcmap = (const uint8_t*)find("pool.cmap")->data;
        DfaPool fp, hp;
        const int32_t* fdesc = (const int32_t*)find("det.first_desc")->data;
        bool fits = true;
        for (int p = 0; p < R.P; ++p) fits &= add_dfa(fp, fdesc + 8 * p, ptrans, pflags, pcmap);
        const int32_t* hdesc = (const int32_t*)find("hot.dfa_desc")->data;
        for (int h = 0; h < R.n_hot; ++h) fits &= add_dfa(hp, hdesc + 8 * h, ptrans, pflags, pcmap);
        if (!fits) return fail("a FIRST/HOT automaton has more than 16384 states");
        if (hp.desc.empty()) hp.desc.assign(8, 0);
        auto vec = [](const auto& v) { return std::make_pair((const void*)v.data(), v.size() * sizeof(v[0])); };
        std::vector<std::pair<const void*, size_t>> pf(FI_N), pe(EV_N), ps(SE_N);
        pf[FI_TRANS] = vec(fp.trans);
        pf[FI_CMAP] = vec(fp.cmap);
        pf[FI_DESC] = vec(fp.desc);
        pe[EV_TRANS] = vec(hp.trans);
        pe[EV_CMAP] = vec(hp.cmap);
        pe[EV_HDESC] = vec(hp.desc);
        pe[EV_HRULE] = sec("hot.rule");
        pe[EV_DTYPE] = sec("det.type");
        pe[EV_DVAL] = sec("det.validator");
        pe[EV_DLIK] = sec("det.lik");
        const size_t n_keys = (size_t)R.V * R.T;
        const ListTab rl = dedup_lists((const uint32_t*)find("var.rule_off")->data,
                                       (const uint16_t*)find("var.rule_ids")->data, n_keys);
        const ListTab xl = dedup_lists((const uint32_t*)find("var.excl_off")->data,
                                       (const uint16_t*)find("var.excl_ids")->data, n_keys);
        const uint32_t aux = rl.w | xl.w << 3;
        e->lists_cl = rl.w != 0 || xl.w != 0;
        pe[EV_ROFF] = vec(rl.ix);
        pe[EV_RLOFF] = vec(rl.loff);
        pe[EV_RIDS] = vec(rl.ids);
        // per type: every hotword rule it has in any context variant (k_win_eval's resident bits)
        std::vector<uint32_t> thot(std::max(R.T, 1), 0u);
        {
            const uint32_t* ro = (const uint32_t*)find("var.rule_off")->data;
            const uint16_t* ri = (const uint16_t*)find("var.rule_ids")->data;
            for (int v = 0; v < R.V; ++v)
                for (int t = 0; t < R.T; ++t)
                    for (uint32_t q = ro[v * R.T + t]; q < ro[v * R.T + t + 1]; ++q)
                        if (ri[q] < 32) thot[t] |= 1u << ri[q];     // k_win_* cache the first WHOT_BITS
        }
        pe[EV_THOT] = vec(thot);
        std::vector<std::pair<const void*, size_t>> pw(WS_N);
        pw[WS_TRANS] = vec(hp.trans);
        pw[WS_CMAP] = vec(hp.cmap);
        pw[WS_HDESC] = vec(hp.desc);
        pw[WS_HRULE] = sec("hot.rule");
        pw[WS_DTYPE] = sec("det.type");
        pw[WS_DLIK] = sec("det.lik");
        pw[WS_VEN] = sec("var.enabled");
        pw[WS_VMIN] = sec("var.minlik");
        pw[WS_DEX] = sec("det.exidx");
        pw[WS_XOFF] = vec(xl.ix);
        pw[WS_XLOFF] = vec(xl.loff);
        pw[WS_XIDS] = vec(xl.ids);
        pw[WS_TOKOFF] = std::make_pair((const void*)tok_off.data(), tok_off.size() * 4);
        pw[WS_ROFF] = vec(rl.ix);
        pw[WS_RLOFF] = vec(rl.loff);
        pw[WS_RIDS] = vec(rl.ids);
        if (!make_image(pw, e->img_wsel)) return fail("rule table upload failed");
        e->img_wsel.li.aux = aux;
        ps[SE_DTYPE] = sec("det.type");
        ps[SE_VEN] = sec("var.enabled");
        ps[SE_VMIN] = sec("var.minlik");
        ps[SE_DEX] = sec("det.exidx");
        ps[SE_XOFF] = vec(xl.ix);
        ps[SE_XLOFF] = vec(xl.loff);
        ps[SE_XIDS] = vec(xl.ids);
        ps[SE_TOKOFF] = std::make_pair((const void*)tok_off.data(), tok_off.size() * 4);
        if (!make_image(pf, e->img_first) || !make_image(pe, e->img_eval) || !make_image(ps, e->img_sel))
            return fail("rule table upload failed");
        e->img_eval.li.aux = aux;
        e->img_sel.li.aux = aux;
        if (e->img_first.global) {
            // FIRST automata for k_pair_first<true>'s LDS copy: patterns in id
            // order (the built-in types first), skipping any automaton over FIRST_HOT_BIG bytes, until
            // the copy is full.  A skipped pattern keeps a descriptor with no columns (read from L2).
            size_t big = FIRST_HOT_BIG, budget = FIRST_HOT_LDS;
            if (const char* v = std::getenv("PII_FIRST_HOT_BIG")) big = (size_t)std::max(0, std::atoi(v));
            if (const char* v = std::getenv("PII_FIRST_HOT_LDS"))
                budget = std::min<size_t>(158 * 1024, (size_t)std::max(0, std::atoi(v)));
            uint32_t cap_p = (uint32_t)R.P;
            if (const char* v = std::getenv("PII_FIRST_HOT")) cap_p = std::min<uint32_t>(cap_p, (uint32_t)std::max(0, std::atoi(v)));
            DfaPool hf;
            uint32_t ph = 0;
            size_t trans_n = 0, cmap_n = 0;
            for (uint32_t p = 0; p < cap_p; ++p) {
                const int32_t* d = fdesc + 8 * p;
                const size_t dfa = (size_t)d[7] * d[3] * 2;
                const size_t tr = trans_n + 64 + (size_t)d[7] * d[3];
                const size_t bytes = ((tr * 2 + 15) & ~(size_t)15) + ((cmap_n + 260 + 15) & ~(size_t)15) +
                                     (((size_t)(p + 1) * 32 + 15) & ~(size_t)15);
                if (bytes > budget) {
                    if (big == 0) break;
                    continue;
                }
                if (big && dfa > big) continue;
                trans_n = tr;
                cmap_n += 260;
                ph = p + 1;
            }
            if (ph > 0) {
                trans_n = 0;
                for (uint32_t p = 0; p < ph; ++p) {
                    const int32_t* d = fdesc + 8 * p;
                    const size_t dfa = (size_t)d[7] * d[3] * 2;
                    const size_t tr = hf.trans.size() + 64 + (size_t)d[7] * d[3];
                    const size_t bytes = ((tr * 2 + 15) & ~(size_t)15) + ((hf.cmap.size() + 260 + 15) & ~(size_t)15) +
                                         (((size_t)ph * 32 + 15) & ~(size_t)15);
                    if ((big && dfa > big) || bytes > budget) {
                        hf.desc.insert(hf.desc.end(), 8, 0);          // columns 0: not resident
                        continue;
                    }
                    add_dfa(hf, d, ptrans, pflags, pcmap);
                }
                std::vector<std::pair<const void*, size_t>> ph_parts(FI_N);
                ph_parts[FI_TRANS] = vec(hf.trans);
                ph_parts[FI_CMAP] = vec(hf.cmap);
                ph_parts[FI_DESC] = vec(hf.desc);
                if (!make_image(ph_parts, e->img_first_hot)) return fail("rule table upload failed");
                if (e->img_first_hot.li.total > 64 * 1024 &&
                    hipFuncSetAttribute((const void*)k_pair_first<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)e->img_first_hot.li.total) != hipSuccess)
                    return fail("cannot raise the LDS limit of k_pair_first");
                e->first_p_hot = ph;
            }
        }
        if (e->img_eval.li.total > IMG_LDS_SPLIT) {
            auto pr = pe;
            pr[EV_ROFF] = std::make_pair((const void*)nullptr, (size_t)0);
            pr[EV_RLOFF] = std::make_pair((const void*)nullptr, (size_t)0);
            pr[EV_RIDS] = std::make_pair((const void*)nullptr, (size_t)0);
            if (!make_image(pr, e->img_eval_rg)) return fail("rule table upload failed");
            if (e->img_eval_rg.global || (e->img_eval_rg.li.total > 64 * 1024 &&
                                          hipFuncSetAttribute((const void*)k_pair_eval<false, true>,
                                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                                              (int)e->img_eval_rg.li.total) != hipSuccess)) {
                (void)hipFree(e->img_eval_rg.d);
                e->img_eval_rg = DevImage{};
            }
        }
        if (e->img_sel.li.total > IMG_LDS_SPLIT) {
            auto pr = ps;
            pr[SE_XOFF] = std::make_pair((const void*)nullptr, (size_t)0);
            pr[SE_XLOFF] = std::make_pair((const void*)nullptr, (size_t)0);
            pr[SE_XIDS] = std::make_pair((const void*)nullptr, (size_t)0);
            if (!make_image(pr, e->img_sel_rg)) return fail("rule table upload failed");
            if (e->img_sel_rg.global || e->img_sel_rg.li.total > 64 * 1024) {      // (no gain: keep the full image)
                (void)hipFree(e->img_sel_rg.d);
                e->img_sel_rg = DevImage{};
            }
        }
        // (the window re-scan's kernels read an image past LDS in place, like the pair kernels)
        const std::pair<const void*, const DevImage*> big[] = {
            {(const void*)k_pair_first<false>, &e->img_first}, {(const void*)k_pair_eval<false>, &e->img_eval},
            {(const void*)k_select<false, false>, &e->img_sel}, {(const void*)k_sel_fix<false, false>, &e->img_sel},
            {(const void*)k_select<false, true>, &e->img_sel}, {(const void*)k_sel_fix<false, true>, &e->img_sel},
            {(const void*)k_select<false, false, true>, &e->img_sel},
            {(const void*)k_sel_fix<false, false, true>, &e->img_sel},
            {(const void*)k_select<false, true, true>, &e->img_sel}, {(const void*)k_sel_fix<false, true, true>, &e->img_sel},
            {(const void*)k_pair_eval<false, false, true>, &e->img_eval},
            {(const void*)k_win_eval<false>, &e->img_eval},
            {(const void*)k_win_select<false>, &e->img_wsel}};
        // k_win_halo<false>: its image plus HALO_LDS of tables (the launch falls back to <true> past the LDS)
        if (hipFuncSetAttribute((const void*)k_win_halo<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)IMG_LDS_MAX) != hipSuccess)
            return fail("cannot raise the LDS limit of k_win_halo");
        for (auto& kb : big)
            if (!kb.second->global && kb.second->li.total > 64 * 1024 &&
                hipFuncSetAttribute(kb.first, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kb.second->li.total) !=
                    hipSuccess)
                return fail("cannot raise the LDS limit of a pair kernel");
        if (const char* v = std::getenv("PII_VERBOSE"); v && std::atoi(v) > 0) {
            const std::pair<const char*, const DevImage*> ims[] = {
                {"first", &e->img_first}, {"first_hot", &e->img_first_hot}, {"eval", &e->img_eval},
                {"eval_rg", &e->img_eval_rg}, {"sel", &e->img_sel}, {"sel_rg", &e->img_sel_rg}, {"wsel", &e->img_wsel}};
            for (auto& im : ims)
                if (im.second->d)
                    std::fprintf(stderr, "pii: image %-9s %8u bytes %s\n", im.first, im.second->li.total,
                                 im.second->global ? "global" : "lds");
        }
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            e->n_cu = prop.multiProcessorCount;
        // k_pair_first: two 1024-thread workgroups per CU, one round (2 or 4 rounds: 160 -> 165 / 164 µs,
        // and k_pair_eval slower on the smaller segments)
        e->n_seg = 2 * (uint32_t)e->n_cu;
        // k_pair_eval work units per k_pair_first workgroup: 2 (config 2: 1 / 2 / 3 / 4 -> 342 / 312 / 315
        // / 318 us); 4 for a large rule set (config 5's longer evaluations: 2 -> 4: 909 -> 893 us)
        if ((size_t)R.V * R.T > LIST_DEDUP_KEYS) e->eval_split = 4;
        if (const char* v = std::getenv("PII_EVAL_SPLIT")) e->eval_split = (uint32_t)std::max(1, std::min(64, std::atoi(v)));
        if (const char* v = std::getenv("PII_MERGE_CAP")) e->merge_cap = (uint32_t)std::max(0, std::min(MERGE_EVW, std::atoi(v)));
        if (hipMalloc(&e->mcount, e->n_seg * PAIR_WAVES * sizeof(uint32_t)) != hipSuccess) return fail("hipMalloc failed");
    }
    e->scan_lds = SCAN_TD_BASE + (size_t)(R.SD * R.CDs / 2) * 4 + (size_t)(R.SK * R.CKs / 2) * 4 + SCAN_SPREAD_BYTES;
    if (e->scan_lds > 160 * 1024) return fail("SCAN tables do not fit in LDS");
    e->n_sg = 1 + (uint32_t)hg.size();
    e->sg.assign(1, R);
    e->sg_lds.assign(1, e->scan_lds);
    e->acct.accid[0] = R.d_accid;
    e->acct.npair[0] = R.d_npair;
    for (size_t q = 0; q < hg.size(); ++q) {
        RulesDev Rq = R;
        const HostGroup& h = hg[q];
        Rq.cmap4 = (const uint32_t*)at(gp[q].cmap);
        Rq.td = (const uint16_t*)at(gp[q].td);
        Rq.tk = (const uint16_t*)at(gp[q].tk);
        Rq.d_accid = (const uint16_t*)at(gp[q].dacc);
        Rq.k_accid = (const uint16_t*)at(gp[q].kacc);
        Rq.d_npair = (const uint16_t*)at(gp[q].npair);
        Rq.SD = h.SD;
        Rq.CD = h.CD;
        Rq.CDs = h.CDs;
        Rq.dsh = h.dsh;
        Rq.d_start = h.start;
        Rq.SK = 1;
        Rq.CK = 2;
        Rq.CKs = 2;
        Rq.k_start = 0;
        e->sg.push_back(Rq);
        e->sg_lds.push_back(h.lds);
        e->acct.accid[q + 1] = Rq.d_accid;
        e->acct.npair[q + 1] = Rq.d_npair;
    }
    const size_t max_lds = *std::max_element(e->sg_lds.begin(), e->sg_lds.end());
    e->max_sg_lds = max_lds;
    {
        std::vector<uint32_t> lds32(e->sg_lds.begin(), e->sg_lds.end());
        if (hipMalloc(&e->d_sg, e->sg.size() * sizeof(RulesDev)) != hipSuccess ||
            hipMalloc(&e->d_sg_lds, lds32.size() * 4) != hipSuccess ||
            hipMemcpy(e->d_sg, e->sg.data(), e->sg.size() * sizeof(RulesDev), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(e->d_sg_lds, lds32.data(), lds32.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            return fail("hipMalloc failed");
    }
    if (const char* v = std::getenv("PII_SCAN2")) e->scan2 = std::atoi(v) != 0;
    if (const char* v = std::getenv("PII_SCAN_ILV")) e->scan_ilv = std::atoi(v) != 0;
    if (const char* v = std::getenv("PII_WIN_LONG")) e->win_long = (uint32_t)std::max(0, std::min(64, std::atoi(v)));
    if (const char* v = std::getenv("PII_HALO_ITEMS")) e->halo_items = (uint32_t)std::max(0, std::min(HALO_ITEMS, std::atoi(v)));
    if (const char* v = std::getenv("PII_TIMING")) e->timing = std::max(0, std::min(2, std::atoi(v)));
    if (max_lds > 64 * 1024 &&
        (hipFuncSetAttribute((const void*)k_scan2<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)max_lds) !=
             hipSuccess ||
         hipFuncSetAttribute((const void*)k_scan2<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)max_lds) !=
             hipSuccess ||
         hipFuncSetAttribute((const void*)k_scan2<false, SCAN_BLOCK_WIDE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)max_lds) != hipSuccess))
        return fail("cannot raise LDS limit");
    if (max_lds > 64 * 1024 &&
        (hipFuncSetAttribute((const void*)k_scan<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)max_lds) !=
             hipSuccess ||
         hipFuncSetAttribute((const void*)k_scan<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)max_lds) !=
             hipSuccess ||
         hipFuncSetAttribute((const void*)k_scan<false, SCAN_BLOCK_WIDE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)max_lds) != hipSuccess ||
         hipFuncSetAttribute((const void*)k_halo, hipFuncAttributeMaxDynamicSharedMemorySize, (int)max_lds) != hipSuccess))
        return fail("cannot raise LDS limit");
    if (max_lds + FIX_LDS > 64 * 1024 &&
        hipFuncSetAttribute((const void*)k_scan_fix, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(max_lds + FIX_LDS)) != hipSuccess)
        return fail("cannot raise LDS limit");
    e->hist_types = (uint32_t)std::min(R.T, 1024);
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    e->own_stream = true;
    if (e->n_sg > 1) {
        int ns_scan = SCAN_STREAMS;
        if (const char* v = std::getenv("PII_SCAN_STREAMS")) ns_scan = std::max(1, std::min(3, std::atoi(v)));
        e->n_aux = (uint32_t)ns_scan - 1;
        if (e->n_aux && hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) != hipSuccess) return fail("event");
        for (uint32_t i = 0; i < e->n_aux; ++i)
            if (hipStreamCreateWithFlags(&e->aux[i], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&e->ev_join[i], hipEventDisableTiming) != hipSuccess)
                return fail("stream");
    }
    for (auto& t : e->kev)
        if (hipEventCreate(&t) != hipSuccess) return fail("event");
    for (auto& t : e->tev)
        if (hipEventCreate(&t) != hipSuccess) return fail("event");
    const size_t ns = std::max<uint32_t>(1, n_conv_slots);
    if (hipMalloc(&e->st_group, ns * 4) != hipSuccess || hipMalloc(&e->st_ts, ns * 8) != hipSuccess ||
        hipMalloc(&e->stamp, ns * 4) != hipSuccess ||
        hipMalloc(&e->d_err, 64) != hipSuccess || hipMalloc(&e->d_totals, hist_bytes(e)) != hipSuccess ||
        hipMalloc(&e->lb_ticket, 32) != hipSuccess ||
        hipMemset(e->lb_ticket, 0, 32) != hipSuccess)
        return fail("state allocation failed");
    e->long_count = e->d_err + 1;
    e->ncommit = e->d_err + 2;
    e->pair_count = reinterpret_cast<unsigned long long*>(e->d_err + 4);
    // the histogram lives right after the totals, so one async copy at the end of a call brings both
    e->hist = reinterpret_cast<unsigned long long*>(e->d_totals + 8);
    if (hipHostMalloc(&e->h_totals, hist_bytes(e)) != hipSuccess) return fail("pinned allocation failed");
    std::vector<int32_t> g(ns, -1);
    if (hipMemcpy(e->st_group, g.data(), ns * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(e->st_ts, 0, ns * 8) != hipSuccess || hipMemset(e->stamp, 0, ns * 4) != hipSuccess ||
        hipMemset(e->hist, 0, std::max(R.T, 256) * 8) != hipSuccess)
        return fail("state init failed");
    k_noop<<<1, 64, 0, e->stream>>>();
    if (hipStreamSynchronize(e->stream) != hipSuccess) return fail("device not usable");
    *out = e;
    return PII_OK;
}

int pii_engine_destroy(pii_engine* e) {
    if (!e) return PII_E_ARG;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    void* ptrs[] = {e->d_rules, e->st_group, e->st_ts, e->stamp, e->ev, e->fd, e->n_ev, e->n_find,
                    e->out_len, e->incl, e->agg_f, e->first_utt, e->lane_perm, e->lane_pos, e->lane_bkt, e->lane_cnt, e->bnd, e->lane_split, e->lane_spl, e->hist_part, e->evloc, e->lane_ev, e->pres, e->pend, e->lane_pair, e->lane_np, e->matched, e->mcount, e->cont,
                    e->img_first.d, e->img_first_hot.d, e->img_eval.d, e->img_eval_rg.d, e->img_sel.d, e->img_sel_rg.d, e->kw, e->ctx, e->agg_v, e->commit,
                    e->span_offs, e->bsum, e->out_offs_tmp, e->lb_state, e->lb_ticket, e->d_err, e->d_totals, e->h_text, e->h_role,
                    e->h_out, e->h_offs, e->h_out_offs, e->h_slot, e->h_ts, e->h_spans, e->h_ctx,
                    e->img_wsel.d, e->wr_desc, e->wr_cnt, e->wr_head, e->wr_arena, e->wc, e->phot, e->wc_first,
                    e->wc_n, e->wbound, e->n_wfind, e->wout_len, e->wfbase, e->wspan_offs, e->wnew, e->wctx, e->wfd,
                    e->long_rows, e->lane_st, e->lane_geo, e->lane_evn, e->lane_nf, e->lane_rd, e->lane_reach, e->lane_rowbase,
                    e->dirty, e->lane_sp, e->spill, e->rsp, e->tile_first, e->h_ext, e->h_ext_n, e->jbuf, e->joff,
                    e->jlen, e->kw2, e->jrole, e->err_saved, e->d_sg, e->d_sg_lds};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (e->h_totals) (void)hipHostFree(e->h_totals);
    if (e->h_jtotal) (void)hipHostFree(e->h_jtotal);
    for (auto& t : e->tev)
        if (t) (void)hipEventDestroy(t);
    for (auto& t : e->kev)
        if (t) (void)hipEventDestroy(t);
    if (e->stream && e->own_stream) (void)hipStreamDestroy(e->stream);
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    for (uint32_t i = 0; i < 2; ++i) {
        if (e->ev_join[i]) (void)hipEventDestroy(e->ev_join[i]);
        if (e->aux[i]) (void)hipStreamDestroy(e->aux[i]);
    }
    delete e;
    return PII_OK;
}

int pii_engine_info(pii_engine* e, pii_info* out) {
    if (!e || !out) return PII_E_ARG;
    out->n_types = (uint32_t)e->R.T;
    out->n_patterns = (uint32_t)e->R.P;
    out->n_context_groups = (uint32_t)e->R.G;
    out->n_conv_slots = e->n_slots;
    out->scan_states_d = (uint32_t)e->R.SD;
    out->scan_states_k = (uint32_t)e->R.SK;
    out->scan_lds_bytes = (uint32_t)e->scan_lds;
    out->reserved = 0;
    return PII_OK;
}

int pii_type_name(pii_engine* e, uint32_t t, char* buf, size_t cap) {
    if (!e || t >= e->names.size()) return PII_E_ARG;
    const std::string& s = e->names[t];
    if (buf && cap) {
        const size_t n = std::min(cap - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int)s.size();
}

int pii_context_group_type(pii_engine* e, uint32_t g) {
    if (!e || g >= e->kw_type.size()) return PII_E_ARG;
    return e->kw_type[g];
}

int pii_scan_redact_device(pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                           const uint32_t* d_slot, const uint8_t* d_role, const int64_t* d_ts, uint8_t* d_out,
                           uint64_t out_cap, uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap,
                           int16_t* d_ctx_info, void* stream) {
    return device_call(e, false, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out, out_cap, d_out_offsets,
                       d_spans, span_cap, d_ctx_info, stream, nullptr);
}

int pii_scan_redact_device_ex(pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                              uint64_t batch_base, uint64_t batch_bytes, const uint32_t* d_slot, const uint8_t* d_role,
                              const int64_t* d_ts, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_offsets,
                              pii_span* d_spans, uint32_t span_cap, int16_t* d_ctx_info, void* stream) {
    const uint64_t decl[2] = {batch_base, batch_bytes};
    return device_call(e, false, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out, out_cap, d_out_offsets,
                       d_spans, span_cap, d_ctx_info, stream, decl);
}

int pii_reserve(pii_engine* e, uint32_t max_utt, uint64_t max_bytes, uint64_t max_out, uint32_t max_spans) {
    if (!e) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    // the most lanes any batch of at most max_bytes can have: big batches take 1 KiB lanes, smaller
    // ones shrink the lanes to keep at least n_cu*256 of them (pick_lane_shift), i.e. < 2*n_cu*256
    const uint32_t sh = pick_lane_shift(e, max_bytes);
    uint64_t lanes = std::max<uint64_t>(((max_bytes + 63) >> sh) + 2, 2ull * e->n_cu * 256 + 2);
    lanes = std::min<uint64_t>(lanes, ((max_bytes + 63) >> MIN_LANE_SHIFT) + 2);
    int rc;
    if ((rc = ensure_scratch(e, max_utt, max_bytes, (uint32_t)std::min<uint64_t>(lanes, 0xffffffffull))) ||
        (rc = ensure_queues(e, max_bytes)) || (rc = ensure_redact(e, max_spans, max_out)))
        return rc;
    if (e->lb_cap < LB_MAX_TILES + 64) {      // the look-back scans' tile states (exclusive_scan: two scans)
        if ((rc = grow(e, e->lb_state, 2 * ((size_t)LB_MAX_TILES + 64)))) return rc;
        HIPCHK(hipMemsetAsync(e->lb_state, 0, 2 * ((size_t)LB_MAX_TILES + 64) * 8, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->lb_cap = LB_MAX_TILES + 64;
    }
    return PII_OK;
}

int pii_sync(pii_engine* e, uint64_t totals[3]) {
    if (!e) return PII_E_ARG;
    HIPCHK(hipEventSynchronize(e->tev[6]));
    for (int attempt = 0; (e->h_totals[2] & ERR_QUEUE) && !(e->h_totals[2] & ERR_ARGS) && attempt < 4; ++attempt) {
        // a work queue overflowed (pair queue, event records, window findings): grow it to the exact
        // need and run the batch again (context and window history were not committed, so the re-run
        // is idempotent)
        const uint64_t need = e->h_totals[3] + 4096, need_ev = e->h_totals[4] + 4096, need_wf = e->h_totals[5] + 4096;
        if (need_ev > e->ev_cap) {
            if (int rc = grow(e, e->evloc, need_ev)) return rc;
            e->ev_cap = need_ev;
        }
        int rc = grow_pairs(e, std::max(need, e->pair_cap));
        if (rc) return rc;
        e->pair_cap = std::max(need, e->pair_cap);
        if (e->last_kind == 1 && need_wf > e->wfd_cap) {
            if ((rc = grow(e, e->wfd, need_wf))) return rc;
            e->wfd_cap = need_wf;
        }
        if ((rc = rerun_last(e))) return rc;
        HIPCHK(hipEventSynchronize(e->tev[6]));
    }
    float tot = 0;
    for (int i = 0; i < 5; ++i) {
        float ms = 0;
        if (e->timing >= 2) HIPCHK(hipEventElapsedTime(&ms, e->tev[i], e->tev[i + 1]));
        e->last_ms[i] = ms;
        tot += ms;
    }
    // (level 1: the call from its start to its completion event, the totals' copy included)
    if (e->timing == 1) HIPCHK(hipEventElapsedTime(&tot, e->tev[0], e->tev[6]));
    e->last_ms[5] = tot;
    e->last_kms[0] = e->last_kms[1] = 0.f;
    if (e->kev_valid && e->timing >= 1) {
        HIPCHK(hipEventElapsedTime(&e->last_kms[0], e->kev[0], e->kev[1]));
        HIPCHK(hipEventElapsedTime(&e->last_kms[1], e->kev[2], e->kev[3]));
    }
    if (totals) {
        totals[0] = e->h_totals[0];
        totals[1] = e->h_totals[1];
        totals[2] = e->h_totals[2];
    }
    const uint64_t f = e->h_totals[2];
    if (f & ERR_ARGS) {
        e->err = "declared batch base / size do not match offsets[0] / offsets[n_utt] - offsets[0]";
        return PII_E_ARG;
    }
    if (f & ERR_SLOT) return PII_E_ARG;
    if (f & ERR_EXT) {
        e->err = "an external span is malformed (start < end <= row length, sorted by start, info_type < n_types, "
                 "likelihood 1..5, ext_n <= ext_stride)";
        return PII_E_ARG;
    }
    if (f & ERR_RING) {
        e->err = "a conversation's re-scan window does not fit its history slot; raise slot_bytes (pii_window_enable)";
        return PII_E_NOMEM;
    }
    if (f & ERR_ORDER) return PII_E_ORDER;
    if (f & ERR_QUEUE) return PII_E_NOMEM;
    if (f & ERR_STITCH) {
        e->err = "internal: a cut row's lanes did not converge";
        return PII_E_DEVICE;
    }
    if (f & ERR_CAPACITY) return PII_E_CAPACITY;
    return PII_OK;
}

int pii_set_timing(pii_engine* e, int level) {
    if (!e || level < 0 || level > 2) return PII_E_ARG;
    HIPCHK(hipStreamSynchronize(e->stream));      // (no call in flight records under the old level)
    e->timing = level;
    return PII_OK;
}

int pii_last_timings(pii_engine* e, float ms[6]) {
    if (!e || !ms) return PII_E_ARG;
    std::memcpy(ms, e->last_ms, sizeof(e->last_ms));
    return PII_OK;
}

int pii_last_queue_sizes(pii_engine* e, uint64_t* pairs, uint64_t* events) {
    if (!e) return PII_E_ARG;
    if (pairs) *pairs = e->h_totals[3];
    if (events) *events = e->h_totals[4];
    return PII_OK;
}

int pii_last_stats(pii_engine* e, uint64_t* out, uint32_t n) {
    if (!e || (!out && n)) return PII_E_ARG;
    const uint64_t all[6] = {e->h_totals[3], e->h_totals[4], e->last_lanes, 1ull << e->lane_shift, e->h_totals[5],
                             e->h_totals[1]};
    for (uint32_t i = 0; i < n && i < 6; ++i) out[i] = all[i];
    return (int)std::min<uint32_t>(n, 6);
}

int pii_last_timings_ex(pii_engine* e, float* ms, uint32_t n) {
    if (!e || (!ms && n)) return PII_E_ARG;
    float all[8];
    std::memcpy(all, e->last_ms, sizeof(e->last_ms));
    all[6] = e->last_kms[0];
    all[7] = e->last_kms[1];
    for (uint32_t i = 0; i < n && i < 8; ++i) ms[i] = all[i];
    return (int)std::min<uint32_t>(n, 8);
}

}  // extern "C"

namespace {
// host-buffer calls: stage the rows through the engine's device buffers, run, wait, copy back
int host_call(pii_engine* e, bool window, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
              const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, uint8_t* out_bytes,
              uint64_t out_cap, uint64_t* out_offsets, pii_span* spans, uint32_t span_cap, uint32_t* n_spans,
              int16_t* ctx_info, const ExtArgs* x = nullptr) {
    if (!e || !offsets || !out_offsets || (n_utt && (!conv_slot || !role))) return PII_E_ARG;
    if (x && (!x->ext || !x->ext_n || x->stride == 0)) return PII_E_ARG;
    for (uint32_t i = 0; i < n_utt; ++i)
        if (offsets[i + 1] < offsets[i]) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    const uint64_t base = offsets[0], total = offsets[n_utt] - base;
    int rc;
    if (total + 16 > e->cap_h_bytes) {
        const uint64_t nb = total + total / 8 + 64;
        if ((rc = grow(e, e->h_text, nb))) return rc;
        e->cap_h_bytes = nb;
    }
    if (n_utt + 1 > e->cap_h_utt) {
        const uint32_t nu = n_utt + n_utt / 8 + 64;
        if ((rc = grow(e, e->h_offs, nu + 1)) || (rc = grow(e, e->h_out_offs, nu + 1)) ||
            (rc = grow(e, e->h_slot, nu)) || (rc = grow(e, e->h_role, nu)) || (rc = grow(e, e->h_ts, nu)) ||
            (rc = grow(e, e->h_ctx, nu)))
            return rc;
        e->cap_h_utt = nu;
    }
    if (out_cap + 16 > e->cap_h_out) {
        const uint64_t nb = out_cap + 64;
        if ((rc = grow(e, e->h_out, nb))) return rc;
        e->cap_h_out = nb;
    }
    if (span_cap + 1 > e->cap_h_spans) {
        const uint32_t ns = span_cap + 64;
        if ((rc = grow(e, e->h_spans, ns))) return rc;
        e->cap_h_spans = ns;
    }
    hipStream_t st = e->stream;
    std::vector<uint64_t> rel(n_utt + 1);
    for (uint32_t i = 0; i <= n_utt; ++i) rel[i] = offsets[i] - base;
    if (total) HIPCHK(hipMemcpyAsync(e->h_text, bytes + base, total, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->h_offs, rel.data(), (n_utt + 1) * 8, hipMemcpyHostToDevice, st));
    if (n_utt) {
        HIPCHK(hipMemcpyAsync(e->h_slot, conv_slot, n_utt * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->h_role, role, n_utt, hipMemcpyHostToDevice, st));
        if (ts_us) HIPCHK(hipMemcpyAsync(e->h_ts, ts_us, n_utt * 8, hipMemcpyHostToDevice, st));
    }
    if (x && n_utt) {          // stage the external spans (stride-padded rows) next to the text
        const uint64_t ne = (uint64_t)n_utt * x->stride;
        if (ne > e->cap_h_ext) {
            if ((rc = grow(e, e->h_ext, ne))) return rc;
            e->cap_h_ext = ne;
        }
        if (n_utt > e->cap_h_ext_n) {
            if ((rc = grow(e, e->h_ext_n, (size_t)n_utt + n_utt / 8 + 64))) return rc;
            e->cap_h_ext_n = n_utt + n_utt / 8 + 64;
        }
        HIPCHK(hipMemcpyAsync(e->h_ext, x->ext, ne * sizeof(pii_span), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->h_ext_n, x->ext_n, (size_t)n_utt * 4, hipMemcpyHostToDevice, st));
    }
    if (window)
        rc = run_window(e, e->h_text, e->h_offs, n_utt, 0, total, e->h_slot, e->h_role, ts_us ? e->h_ts : nullptr,
                        e->h_out, out_cap, e->h_out_offs, e->h_spans, span_cap, e->h_ctx, st);
    else
        rc = run_pipeline(e, e->h_text, e->h_offs, n_utt, 0, total, e->h_slot, e->h_role, ts_us ? e->h_ts : nullptr,
                          e->h_out, out_cap, e->h_out_offs, e->h_spans, span_cap, e->h_ctx, st,
                          x ? e->h_ext : nullptr, x ? e->h_ext_n : nullptr, x ? x->stride : 0);
    if (rc) return rc;
    uint64_t tot[3];
    rc = pii_sync(e, tot);
    if (rc == PII_E_CAPACITY) {
        HIPCHK(hipMemcpy(out_offsets, e->h_out_offs, (n_utt + 1) * 8, hipMemcpyDeviceToHost));
        if (n_spans) *n_spans = (uint32_t)tot[1];
        return rc;
    }
    if (rc) return rc;
    HIPCHK(hipMemcpy(out_offsets, e->h_out_offs, (n_utt + 1) * 8, hipMemcpyDeviceToHost));
    if (tot[0]) HIPCHK(hipMemcpy(out_bytes, e->h_out, tot[0], hipMemcpyDeviceToHost));
    if (tot[1]) HIPCHK(hipMemcpy(spans, e->h_spans, tot[1] * sizeof(pii_span), hipMemcpyDeviceToHost));
    if (n_spans) *n_spans = (uint32_t)tot[1];
    if (ctx_info && n_utt) HIPCHK(hipMemcpy(ctx_info, e->h_ctx, n_utt * 2, hipMemcpyDeviceToHost));
    return PII_OK;
}

// pii_context_update: stage the rows as host_call does, run the context-only pipeline, copy ctx_info back
int host_context(pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                 const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, int16_t* ctx_info) {
    if (!e || !offsets || (n_utt && (!conv_slot || !role))) return PII_E_ARG;
    for (uint32_t i = 0; i < n_utt; ++i)
        if (offsets[i + 1] < offsets[i]) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    const uint64_t base = offsets[0], total = offsets[n_utt] - base;
    int rc;
    if (total + 16 > e->cap_h_bytes) {
        const uint64_t nb = total + total / 8 + 64;
        if ((rc = grow(e, e->h_text, nb))) return rc;
        e->cap_h_bytes = nb;
    }
    if (n_utt + 1 > e->cap_h_utt) {
        const uint32_t nu = n_utt + n_utt / 8 + 64;
        if ((rc = grow(e, e->h_offs, nu + 1)) || (rc = grow(e, e->h_out_offs, nu + 1)) ||
            (rc = grow(e, e->h_slot, nu)) || (rc = grow(e, e->h_role, nu)) || (rc = grow(e, e->h_ts, nu)) ||
            (rc = grow(e, e->h_ctx, nu)))
            return rc;
        e->cap_h_utt = nu;
    }
    hipStream_t st = e->stream;
    std::vector<uint64_t> rel(n_utt + 1);
    for (uint32_t i = 0; i <= n_utt; ++i) rel[i] = offsets[i] - base;
    if (total) HIPCHK(hipMemcpyAsync(e->h_text, bytes + base, total, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->h_offs, rel.data(), (n_utt + 1) * 8, hipMemcpyHostToDevice, st));
    if (n_utt) {
        HIPCHK(hipMemcpyAsync(e->h_slot, conv_slot, n_utt * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->h_role, role, n_utt, hipMemcpyHostToDevice, st));
        if (ts_us) HIPCHK(hipMemcpyAsync(e->h_ts, ts_us, n_utt * 8, hipMemcpyHostToDevice, st));
    }
    if ((rc = run_context(e, e->h_text, e->h_offs, n_utt, total, e->h_slot, e->h_role, ts_us ? e->h_ts : nullptr,
                          e->h_ctx, st)))
        return rc;
    if ((rc = pii_sync(e, nullptr))) return rc;
    if (ctx_info && n_utt) HIPCHK(hipMemcpy(ctx_info, e->h_ctx, n_utt * 2, hipMemcpyDeviceToHost));
    return PII_OK;
}

int device_call(pii_engine* e, bool window, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                const uint32_t* d_slot, const uint8_t* d_role, const int64_t* d_ts, uint8_t* d_out, uint64_t out_cap,
                uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap, int16_t* d_ctx_info, void* stream,
                const uint64_t* declared, const ExtArgs* x) {
    if (!e || !d_offsets || !d_slot || !d_role || !d_out_offsets) return PII_E_ARG;
    if (n_utt > 0 && (!d_bytes || !d_out || !d_spans)) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : e->stream;
    uint64_t tb[2] = {0, 0};
    if (declared) {          // the caller states offsets[0] and the batch size: no host round trip
        tb[0] = declared[0];
        tb[1] = declared[0] + declared[1];
    } else {
        HIPCHK(hipMemcpyAsync(tb, d_offsets, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(tb + 1, d_offsets + n_utt, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    if (tb[1] < tb[0]) return PII_E_ARG;
    if (window)
        return run_window(e, d_bytes, d_offsets, n_utt, tb[0], tb[1] - tb[0], d_slot, d_role, d_ts, d_out, out_cap,
                          d_out_offsets, d_spans, span_cap, d_ctx_info, st);
    return run_pipeline(e, d_bytes, d_offsets, n_utt, tb[0], tb[1] - tb[0], d_slot, d_role, d_ts, d_out, out_cap,
                        d_out_offsets, d_spans, span_cap, d_ctx_info, st, x ? x->ext : nullptr, x ? x->ext_n : nullptr,
                        x ? x->stride : 0);
}
}  // namespace

extern "C" {

int pii_scan_redact(pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                    const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, uint8_t* out_bytes,
                    uint64_t out_cap, uint64_t* out_offsets, pii_span* spans, uint32_t span_cap, uint32_t* n_spans,
                    int16_t* ctx_info) {
    return host_call(e, false, bytes, offsets, n_utt, conv_slot, role, ts_us, out_bytes, out_cap, out_offsets, spans,
                     span_cap, n_spans, ctx_info);
}

int pii_context_update(pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                       const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, int16_t* ctx_info) {
    return host_context(e, bytes, offsets, n_utt, conv_slot, role, ts_us, ctx_info);
}

int pii_scan_redact_ext(pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                        const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, uint8_t* out_bytes,
                        uint64_t out_cap, uint64_t* out_offsets, pii_span* spans, uint32_t span_cap, uint32_t* n_spans,
                        int16_t* ctx_info, const pii_span* ext, const uint32_t* ext_n, uint32_t ext_stride) {
    const ExtArgs x{ext, ext_n, ext_stride};
    return host_call(e, false, bytes, offsets, n_utt, conv_slot, role, ts_us, out_bytes, out_cap, out_offsets, spans,
                     span_cap, n_spans, ctx_info, &x);
}

int pii_scan_redact_device_ext(pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                               uint64_t batch_base, uint64_t batch_bytes, const uint32_t* d_slot, const uint8_t* d_role,
                               const int64_t* d_ts, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_offsets,
                               pii_span* d_spans, uint32_t span_cap, int16_t* d_ctx_info, const pii_span* d_ext,
                               const uint32_t* d_ext_n, uint32_t ext_stride, void* stream) {
    if (!d_ext || !d_ext_n || ext_stride == 0) return PII_E_ARG;
    const uint64_t decl[2] = {batch_base, batch_bytes};
    const ExtArgs x{d_ext, d_ext_n, ext_stride};
    return device_call(e, false, d_bytes, d_offsets, n_utt, d_slot, d_role, d_ts, d_out, out_cap, d_out_offsets,
                       d_spans, span_cap, d_ctx_info, stream, decl, &x);
}

int pii_window_enable_ex(pii_engine* e, uint32_t window_n, uint32_t slot_bytes, uint32_t flags) {
    if (!e || window_n == 0 || window_n > WN_MAX || slot_bytes < 64 || slot_bytes % 16 ||
        (flags & ~(uint32_t)PII_WINDOW_FULL))
        return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    // the history rings are persistent state like the context table (not work buffers: they do not
    // count against pii_set_scratch_limit); a failed allocation leaves the previous window, if any,
    // enabled and unchanged
    const size_t ns = std::max<uint32_t>(1, e->n_slots);
    WinTables w;
    int rc = alloc_window_tables(e, w, ns, window_n, slot_bytes);
    if (rc) return rc;
    free_window_tables(e);
    e->wr_desc = w.desc;
    e->wr_cnt = w.cnt;
    e->wr_head = w.head;
    e->wr_arena = w.arena;
    // the incremental path needs no detector that consumes '\n' or tests a text edge (a match inside a
    // window is then its utterance's own match); it takes any number of patterns and SCAN groups
    // (config 5: the groups' merged pair queue, candidate lists past LIVE patterns spilled like
    // k_select's) and tables past LDS (read in place); any other rule set re-scans the joined windows
    // in full
    e->win_full = (flags & PII_WINDOW_FULL) || !e->window_ok;
    e->win_n = window_n;
    e->win_slot_bytes = slot_bytes;
    return PII_OK;
}

int pii_context_resize(pii_engine* e, uint32_t n_conv_slots) {
    if (!e || n_conv_slots < e->n_slots) return PII_E_ARG;
    if (n_conv_slots == e->n_slots) return PII_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const size_t ns = n_conv_slots, old = std::max<uint32_t>(1, e->n_slots);
    int32_t* g = nullptr;
    int64_t* t = nullptr;
    uint32_t* s = nullptr;
    auto undo = [&](int rc) {
        if (g) (void)hipFree(g);
        if (t) (void)hipFree(t);
        if (s) (void)hipFree(s);
        (void)hipGetLastError();
        e->err = "device allocation failed: the context table could not grow";
        return rc;
    };
    if (hipMalloc(&g, ns * 4) != hipSuccess || hipMalloc(&t, ns * 8) != hipSuccess || hipMalloc(&s, ns * 4) != hipSuccess)
        return undo(PII_E_NOMEM);
    WinTables w;
    if (e->win_n) {
        const int rc = alloc_window_tables(e, w, ns, e->win_n, e->win_slot_bytes);
        if (rc) return undo(rc);
    }
    // new slots: no context record, no window history; old slots keep theirs (slot-major layouts)
    std::vector<int32_t> none(ns - old, -1);
    bool ok = hipMemcpy(g, e->st_group, old * 4, hipMemcpyDeviceToDevice) == hipSuccess &&
              hipMemcpy(g + old, none.data(), (ns - old) * 4, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(t, e->st_ts, old * 8, hipMemcpyDeviceToDevice) == hipSuccess &&
              hipMemset(t + old, 0, (ns - old) * 8) == hipSuccess &&
              hipMemcpy(s, e->stamp, old * 4, hipMemcpyDeviceToDevice) == hipSuccess &&
              hipMemset(s + old, 0, (ns - old) * 4) == hipSuccess;
    if (ok && e->win_n) {
        const size_t N = e->win_n, sb = e->win_slot_bytes;
        ok = hipMemcpy(w.desc, e->wr_desc, old * N * sizeof(WDesc), hipMemcpyDeviceToDevice) == hipSuccess &&
             hipMemcpy(w.cnt, e->wr_cnt, old * 4, hipMemcpyDeviceToDevice) == hipSuccess &&
             hipMemcpy(w.head, e->wr_head, old * 4, hipMemcpyDeviceToDevice) == hipSuccess &&
             hipMemcpy(w.arena, e->wr_arena, old * sb, hipMemcpyDeviceToDevice) == hipSuccess;
    }
    if (!ok) {
        if (e->win_n) {
            (void)hipFree(w.desc);
            (void)hipFree(w.cnt);
            (void)hipFree(w.head);
            (void)hipFree(w.arena);
        }
        return undo(PII_E_DEVICE);
    }
    (void)hipFree(e->st_group);
    (void)hipFree(e->st_ts);
    (void)hipFree(e->stamp);
    e->st_group = g;
    e->st_ts = t;
    e->stamp = s;
    if (e->win_n) {
        free_window_tables(e);
        e->wr_desc = w.desc;
        e->wr_cnt = w.cnt;
        e->wr_head = w.head;
        e->wr_arena = w.arena;
    }
    e->n_slots = n_conv_slots;
    return PII_OK;
}

int pii_window_enable(pii_engine* e, uint32_t window_n, uint32_t slot_bytes) {
    return pii_window_enable_ex(e, window_n, slot_bytes, 0);
}

int pii_set_scratch_limit(pii_engine* e, uint64_t bytes) {
    if (!e) return PII_E_ARG;
    e->scratch_limit = bytes;
    return PII_OK;
}

int pii_scratch_bytes(pii_engine* e, uint64_t* used) {
    if (!e || !used) return PII_E_ARG;
    *used = e->scratch_used;
    return PII_OK;
}

int pii_window_mode(pii_engine* e) {
    if (!e || e->win_n == 0) return PII_E_ARG;
    return e->win_full ? PII_WINDOW_FULL : 0;
}

int pii_window_reset(pii_engine* e, uint32_t slot) {
    if (!e || e->win_n == 0 || slot >= e->n_slots) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const uint32_t z = 0;
    HIPCHK(hipMemcpy(e->wr_cnt + slot, &z, 4, hipMemcpyHostToDevice));
    return PII_OK;
}

int pii_window_count(pii_engine* e, uint32_t slot, uint32_t* n_entries) {
    if (!e || e->win_n == 0 || slot >= e->n_slots || !n_entries) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(n_entries, e->wr_cnt + slot, 4, hipMemcpyDeviceToHost));
    return PII_OK;
}

int pii_rescan_window(pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                      const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, uint8_t* out_bytes,
                      uint64_t out_cap, uint64_t* out_offsets, pii_span* spans, uint32_t span_cap, uint32_t* n_spans,
                      int16_t* win_ctx) {
    return host_call(e, true, bytes, offsets, n_utt, conv_slot, role, ts_us, out_bytes, out_cap, out_offsets, spans,
                     span_cap, n_spans, win_ctx);
}

int pii_rescan_window_device(pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                             const uint32_t* d_conv_slot, const uint8_t* d_role, const int64_t* d_ts_us,
                             uint8_t* d_out_bytes, uint64_t out_cap, uint64_t* d_out_offsets, pii_span* d_spans,
                             uint32_t span_cap, int16_t* d_win_ctx, void* stream) {
    return device_call(e, true, d_bytes, d_offsets, n_utt, d_conv_slot, d_role, d_ts_us, d_out_bytes, out_cap,
                       d_out_offsets, d_spans, span_cap, d_win_ctx, stream, nullptr);
}

int pii_rescan_window_device_ex(pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                                uint64_t batch_base, uint64_t batch_bytes, const uint32_t* d_conv_slot,
                                const uint8_t* d_role, const int64_t* d_ts_us, uint8_t* d_out_bytes, uint64_t out_cap,
                                uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap, int16_t* d_win_ctx,
                                void* stream) {
    const uint64_t decl[2] = {batch_base, batch_bytes};
    return device_call(e, true, d_bytes, d_offsets, n_utt, d_conv_slot, d_role, d_ts_us, d_out_bytes, out_cap,
                       d_out_offsets, d_spans, span_cap, d_win_ctx, stream, decl);
}

int pii_context_get(pii_engine* e, uint32_t slot, int32_t* group, int64_t* ts_us) {
    if (!e || slot >= e->n_slots) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    int32_t g;
    int64_t t;
    HIPCHK(hipMemcpy(&g, e->st_group + slot, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&t, e->st_ts + slot, 8, hipMemcpyDeviceToHost));
    if (group) *group = g;
    if (ts_us) *ts_us = t;
    return PII_OK;
}

int pii_context_set(pii_engine* e, uint32_t slot, int32_t group, int64_t ts_us) {
    if (!e || slot >= e->n_slots || group < -1 || group >= e->R.G) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(e->st_group + slot, &group, 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->st_ts + slot, &ts_us, 8, hipMemcpyHostToDevice));
    return PII_OK;
}

int pii_histogram(pii_engine* e, uint64_t* counts, uint32_t n) {
    if (!e || !counts) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    const uint32_t T = (uint32_t)e->R.T;
    if (e->hist_zero_pending) {    // reset since the last call: the next call zeroes the device copy
        for (uint32_t i = 0; i < n; ++i) counts[i] = 0;
        return PII_OK;
    }
    if (e->h_hist_valid) {         // the last call copied it with its totals: no extra round trip
        HIPCHK(hipEventSynchronize(e->tev[6]));
        const uint64_t* h = e->h_totals + 8;
        for (uint32_t i = 0; i < n; ++i) counts[i] = i < T ? h[i] : 0;
        return PII_OK;
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    std::vector<unsigned long long> h(T);
    if (T) HIPCHK(hipMemcpy(h.data(), e->hist, T * 8, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) counts[i] = i < T ? h[i] : 0;
    return PII_OK;
}

// deferred: the next call's first kernel (k_begin) zeroes the histogram on that call's stream, after
// the previous call (calls are sequential: each is followed by pii_sync); until then pii_histogram
// reports zeros.  No device command and no host wait here.
int pii_histogram_reset(pii_engine* e) {
    if (!e) return PII_E_ARG;
    e->h_hist_valid = false;
    e->hist_zero_pending = true;
    return PII_OK;
}

}  // extern "C"
