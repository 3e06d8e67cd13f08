/*
 * pii_engine.h - C ABI of the MI355X PII scan-and-redact engine (libpii.so).
 *
 * Drop-in boundary for the de-identification step of iyngr/context-based-pii:
 *
 *   main_service/main.py:580  call_dlp_for_redaction(transcript, context) -> str
 *       builds a DLP request (main.py:596-726) and calls
 *   main_service/main.py:728  dlp_client.deidentify_content(request=...)
 *
 * The engine replaces the remote DLP call AND the Redis context record the handlers keep
 * (main.py:366-374 SETEX context:{conversation_id}, TTL CONTEXT_TTL_SECONDS=90, main.py:163;
 * GET at main.py:403/444): per-conversation context lives in HBM, indexed by a caller-chosen
 * conversation SLOT (the Python shim maps conversation_id strings to slots).
 *
 * One engine per GPU; calls on one engine are serialised by the caller (not re-entrant), exactly
 * like one gunicorn worker's DLP client (main_service/Dockerfile:29).  Plain pointers and sizes only.
 *
 * Batch contract (pii_scan_redact*): rows are utterances in arrival order.  Rows of one
 * conversation must be contiguous in the batch and in original_entry_index order (the replay /
 * ingest order); a slot that appears in two separate runs of one batch is rejected with
 * PII_E_ORDER.  AGENT rows are redacted without context and then update their conversation's
 * context from the context keywords (handle_agent_utterance, main.py:344-384); CUSTOMER rows are
 * redacted with the conversation's live context (handle_customer_utterance, main.py:386-425);
 * OTHER rows are redacted without context and leave it unchanged.
 */
#ifndef PII_ENGINE_H
#define PII_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes; the Python shim maps them onto the reference's error strings
 * ([DLP_PROCESSING_ERROR] {transcript} ..., main.py:752-773) */
#define PII_OK 0
/* largest batch (sum of row bytes) one call accepts: event/pair positions are 32-bit */
#define PII_MAX_BATCH_BYTES 0xFFFF0000ull

#define PII_E_ARG -1       /* bad argument / malformed offsets                              */
#define PII_E_RULES -2     /* rules blob malformed or unsupported                           */
#define PII_E_DEVICE -3    /* HIP runtime error                                             */
#define PII_E_CAPACITY -4  /* out_cap or span_cap too small: required sizes written back    */
#define PII_E_ORDER -5     /* a conversation slot appears in two runs of one batch          */
#define PII_E_NOMEM -6     /* device allocation failed                                      */

#define PII_ROLE_CUSTOMER 0 /* END_USER / CUSTOMER (subscriber_service/main.py:229) */
#define PII_ROLE_AGENT 1    /* AGENT (subscriber_service/main.py:200)              */
#define PII_ROLE_OTHER 2

/* one kept finding: byte offsets into the UTF-8 input of row `utt` */
typedef struct pii_span {
    uint32_t utt;
    uint32_t start;
    uint32_t end;
    uint16_t info_type;  /* index into the engine's type table (pii_type_name) */
    uint8_t likelihood;  /* DLP scale: 1 VERY_UNLIKELY .. 5 VERY_LIKELY         */
    uint8_t flags;
} pii_span;

typedef struct pii_info {
    uint32_t n_types;          /* info types (YAML info_types, custom types, build-defined)  */
    uint32_t n_patterns;       /* detector patterns                                          */
    uint32_t n_context_groups; /* context_keywords groups (dlp_config.yaml:5-91)              */
    uint32_t n_conv_slots;
    uint32_t scan_states_d;    /* SCAN prefilter automaton states                             */
    uint32_t scan_states_k;    /* context-keyword automaton states                            */
    uint32_t scan_lds_bytes;   /* LDS the scan kernel needs per workgroup                     */
    uint32_t reserved;
} pii_info;

/* Rules blob = output of context-based-pii_amd/compiler.py (compiled dlp_config.yaml).
 * Replaces: the DLP inspect/deidentify templates (deployment/update_dlp_templates.py:38-78). */
int pii_engine_create(const void* rules_blob, size_t blob_bytes, int device, uint32_t n_conv_slots,
                      int64_t context_ttl_us, struct pii_engine** out);
int pii_engine_destroy(struct pii_engine* e);
int pii_engine_info(struct pii_engine* e, pii_info* out);
/* name of info type `t` ("CREDIT_CARD_NUMBER"); returns its length or a negative error */
int pii_type_name(struct pii_engine* e, uint32_t t, char* buf, size_t cap);
/* name of the context group `g` (its expected_pii_type) */
int pii_context_group_type(struct pii_engine* e, uint32_t g);
const char* pii_last_error(struct pii_engine* e);

/* Host-buffer entry point (replaces call_dlp_for_redaction for a batch of transcripts).
 *   bytes/offsets : n_utt rows, row i = bytes[offsets[i] .. offsets[i+1])
 *   conv_slot     : conversation slot per row (< n_conv_slots)
 *   role          : PII_ROLE_* per row
 *   ts_us         : per-row timestamp (start_timestamp_usec) for the context TTL; NULL = no expiry
 *   out_bytes     : redacted rows, packed; out_offsets[n_utt+1]
 *   spans         : kept findings ordered by (utt, start); *n_spans = count
 *   ctx_info      : optional int16[n_utt]: AGENT rows -> context group stored (-1 none),
 *                   CUSTOMER rows -> context group used (-1 none), OTHER -> -1
 * On PII_E_CAPACITY, out_offsets[n_utt] = required bytes and *n_spans = required spans, and the
 * conversation context is NOT updated (the call can be retried). */
int pii_scan_redact(struct pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                    const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us,
                    uint8_t* out_bytes, uint64_t out_cap, uint64_t* out_offsets,
                    pii_span* spans, uint32_t span_cap, uint32_t* n_spans, int16_t* ctx_info);

/* Device-buffer entry point: every pointer is device memory (inputs already resident in HBM).
 * Work is enqueued on `stream` (NULL = the engine's stream) and returns without waiting; call
 * pii_sync() for the totals.  d_bytes is read in aligned 16-byte chunks that stay inside
 * [d_bytes, d_bytes + offsets[n_utt]). */
int pii_scan_redact_device(struct pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets,
                           uint32_t n_utt, const uint32_t* d_conv_slot, const uint8_t* d_role,
                           const int64_t* d_ts_us, uint8_t* d_out_bytes, uint64_t out_cap,
                           uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap,
                           int16_t* d_ctx_info, void* stream);
/* The same call with the batch's offsets[0] (batch_base) and byte size (offsets[n_utt] - offsets[0])
 * stated by the caller, so that enqueueing it needs no device-to-host read (pii_scan_redact_device
 * reads the two offsets back and waits for them).  A streaming ingest (config 4: the reference's
 * Pub/Sub -> subscriber -> handler chain, main_service/main.py:522-562 -> :386-425 -> :580, one DLP
 * RPC per message) enqueues batch i+1 while batch i's output is still being copied out.  A wrong
 * declaration is detected on the device and pii_sync() returns PII_E_ARG; nothing is committed. */
int pii_scan_redact_device_ex(struct pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets,
                              uint32_t n_utt, uint64_t batch_base, uint64_t batch_bytes,
                              const uint32_t* d_conv_slot, const uint8_t* d_role, const int64_t* d_ts_us,
                              uint8_t* d_out_bytes, uint64_t out_cap, uint64_t* d_out_offsets,
                              pii_span* d_spans, uint32_t span_cap, int16_t* d_ctx_info, void* stream);
/* External candidates: the findings of a detector outside the rules blob -- the
 * optional NER (libner.so, ner.py) and its PERSON_NAME, the detector the "full name|your name" hotword
 * of main_service/dlp_config.yaml:170 asks for and no configured detector provides.  Row i's
 * candidates are ext[i * ext_stride + k] for k < ext_n[i] (<= ext_stride): start / end row-relative
 * byte offsets, sorted by start, info_type < n_types (normally one of the rules' external types,
 * rules/builtin_infotypes.yaml `external_types`), likelihood 1..5; utt and flags are ignored.  They
 * join the rule findings in overlap resolution -- after validation and hotwords, subject
 * to min_likelihood and the context variant's enabled types, never as excluders -- so they reach the
 * span list, the redacted bytes ("[PERSON_NAME]") and the histogram like any finding.  A malformed
 * span fails the call with PII_E_ARG (nothing committed).  Otherwise identical to
 * pii_scan_redact / pii_scan_redact_device_ex. */
int pii_scan_redact_ext(struct pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                        const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us,
                        uint8_t* out_bytes, uint64_t out_cap, uint64_t* out_offsets,
                        pii_span* spans, uint32_t span_cap, uint32_t* n_spans, int16_t* ctx_info,
                        const pii_span* ext, const uint32_t* ext_n, uint32_t ext_stride);
int pii_scan_redact_device_ext(struct pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets,
                               uint32_t n_utt, uint64_t batch_base, uint64_t batch_bytes,
                               const uint32_t* d_conv_slot, const uint8_t* d_role, const int64_t* d_ts_us,
                               uint8_t* d_out_bytes, uint64_t out_cap, uint64_t* d_out_offsets,
                               pii_span* d_spans, uint32_t span_cap, int16_t* d_ctx_info,
                               const pii_span* d_ext, const uint32_t* d_ext_n, uint32_t ext_stride, void* stream);
/* Pre-size every internal work buffer for batches of at most max_utt rows / max_bytes input bytes /
 * max_out output bytes / max_spans spans, so that calls within those bounds allocate nothing (no
 * hipMalloc, which synchronizes the device, inside a streaming loop).  The pair / event queues still
 * grow on overflow (pii_sync re-runs the batch) -- their need depends on the text, not its size. */
int pii_reserve(struct pii_engine* e, uint32_t max_utt, uint64_t max_bytes, uint64_t max_out, uint32_t max_spans);
/* Bound the device memory of the engine's per-call work buffers (queues, arenas, staging; not the rules
 * or the persistent context / window tables, which pii_engine_create, pii_window_enable and
 * pii_context_resize allocate outside it), e.g. on a GPU shared with other work; 0 = no limit.  A call that
 * would need more fails with PII_E_NOMEM and commits nothing (the service maps it to
 * "[DLP_PROCESSING_ERROR] {transcript}", main.py:770-773); buffers already held stay valid.
 * pii_scratch_bytes reports what the work buffers hold now.  A growing buffer is allocated before the
 * old one is freed (a failed growth leaves the engine usable), so growing one of the large arenas
 * needs its old and new size at once for a moment; pii_reserve up front avoids growth in the loop. */
int pii_set_scratch_limit(struct pii_engine* e, uint64_t bytes);
int pii_scratch_bytes(struct pii_engine* e, uint64_t* used);
/* wait for the last device call; totals[0] = output bytes, [1] = spans, [2] = error flags */
int pii_sync(struct pii_engine* e, uint64_t totals[3]);

/* per-conversation context record (replaces redis GET/SETEX of context:{id}) */
int pii_context_get(struct pii_engine* e, uint32_t slot, int32_t* group, int64_t* ts_us);
int pii_context_set(struct pii_engine* e, uint32_t slot, int32_t group, int64_t ts_us);
/* Grow the conversation table to n_conv_slots (>= the current count; PII_E_ARG otherwise).  Redis
 * keeps every context:{id} key until its TTL runs out (main.py:163, 366-374), so the host slot map
 * grows the table instead of evicting a conversation whose record is still live.  Records and
 * window histories of the existing slots are kept; new slots start empty.  Synchronous.  On failure
 * (PII_E_NOMEM) the table is unchanged.  Peak device memory: the new tables are allocated and filled
 * before the old ones are freed, so the call briefly holds old + new = (n_old + n_conv_slots) x
 * (16 B of context record + with the window enabled, window_n x 16 B of ring entries + 8 B of ring
 * counters + slot_bytes of ring text) -- e.g. doubling 64k slots with N = 5 and 8 KiB rings holds
 * about 1.6 GB at once.  The service answers a failed growth with the reference's error string
 * for that conversation (service.SlotMap, "[DLP_PROCESSING_ERROR] {transcript}"). */
int pii_context_resize(struct pii_engine* e, uint32_t n_conv_slots);
/* The context half of pii_scan_redact alone, for rows whose redaction failed: the reference stores
 * an agent utterance's context even when its DLP call failed (call_dlp_for_redaction never raises;
 * extract_expected_pii + SETEX run after it, main.py:358-374).  Same batch contract and context
 * semantics (AGENT rows' keyword hits are committed, ctx_info as in pii_scan_redact: an AGENT row's
 * own group, else the record the row read); no findings, no output, no histogram.  Needs the scan's
 * work buffers but no pair queue, so it fits where a full call may not. */
int pii_context_update(struct pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                       const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, int16_t* ctx_info);

/* per-info-type counts of kept findings since the last reset (counts[n_types]); the multi-GPU
 * driver all-reduces these over RCCL.  Each call copies the counts to pinned host memory with its
 * totals, so reading them after pii_sync costs no further device round trip.  The reset issues no
 * device command: the next call's first kernel zeroes the counts (on that call's stream), and until
 * that call pii_histogram reports zeros. */
int pii_histogram(struct pii_engine* e, uint64_t* counts, uint32_t n);
int pii_histogram_reset(struct pii_engine* e);

/* what a call records with HIP events on its stream: 0 = its completion only; 1 (default) = + its
 * start and the events around the scan and redaction kernels; 2 = + the stage boundaries.  An event
 * between two kernels costs the stream a few microseconds, so level 2 is for profiling runs.
 * (env PII_TIMING sets the default; the call waits for the engine stream) */
int pii_set_timing(struct pii_engine* e, int level);
/* per-stage device time of the last call, milliseconds (HIP events on the engine stream):
 * [0] scan [1] context [2] resolve [3] offsets [4] redact (timing level 2; 0 below) [5] total
 * (level >= 1) */
int pii_last_timings(struct pii_engine* e, float ms[6]);
/* the same six, then [6] the reverse DFA scan kernel (k_scan) and [7] the redaction kernel
 * (k_redact) alone; fills min(n, 8) entries and returns that count */
int pii_last_timings_ex(struct pii_engine* e, float* ms, uint32_t n);
/* sizes of the last call's internal work queues: (start, pattern) candidate pairs and SCAN events
 * (what the roofline accounting of k_scan counts as written) */
int pii_last_queue_sizes(struct pii_engine* e, uint64_t* pairs, uint64_t* events);
/* the last call's work sizes: [0] candidate pairs [1] scan events [2] scan lanes [3] bytes per scan lane
 * (1 KiB for big batches, down to 128 B for small ones) [4] window-findings arena entries [5] spans;
 * fills min(n, 6) entries and returns that count */
int pii_last_stats(struct pii_engine* e, uint64_t* out, uint32_t n);

/* ---------------------------------------------------------------- multi-turn window re-scan (a12)
 * Replaces the aggregator's sliding-window re-scan (README.md:131-134, 159-168: keep the last N
 * utterances of a conversation -- N = 5, transcript_aggregator_service/cloudbuild.yaml:33 -- join
 * them with "\n" and send the joined text through handle_customer_utterance, main.py:386-425) and
 * the Redis list that held the window.  The window history lives in HBM per conversation slot
 * (`slot_bytes` each) and keeps, per utterance, its text and its resident detector candidates, so a
 * re-scan scans only the NEW utterance; the rest of the window costs a hotword re-check where a
 * proximity window crosses a "\n", the context variant, and the output copy.  Output per row =
 * redact("\n".join(window ending at that row), current expected_pii_type) bit-exactly (SURVEY A.9,
 * oracle/pii_oracle.py window_rescan), for every rule set: when no detector can match '\n' or a text
 * edge, incrementally (the shipped rules and config-5 scale rule sets alike: any number of patterns
 * and SCAN groups, tables in LDS or read in place); otherwise (a '\n'-consuming detector) by a FULL
 * re-scan -- the ring then keeps the raw text, every row's "\n"-joined window is materialised in HBM
 * and run through the scan+redact pipeline (one host wait per call for the joined size). */
#define PII_WINDOW_MAX 8
#define PII_WINDOW_FULL 1   /* pii_window_enable_ex flag / pii_window_mode result: full re-scan */
/* allocate the per-slot window history (n_conv_slots * slot_bytes of HBM); window_n <= PII_WINDOW_MAX,
 * slot_bytes a multiple of 16 (a window must fit: its utterances + 16 B per resident candidate) */
int pii_window_enable(struct pii_engine* e, uint32_t window_n, uint32_t slot_bytes);
/* the same; flags PII_WINDOW_FULL forces the full re-scan even for rules the incremental path takes */
int pii_window_enable_ex(struct pii_engine* e, uint32_t window_n, uint32_t slot_bytes, uint32_t flags);
/* PII_WINDOW_FULL or 0 (incremental) for an enabled window, else PII_E_ARG */
int pii_window_mode(struct pii_engine* e);
/* forget a conversation's window (the /conversation-ended endpoint, aggregator main.py) */
int pii_window_reset(struct pii_engine* e, uint32_t slot);
int pii_window_count(struct pii_engine* e, uint32_t slot, uint32_t* n_entries);
/* Batch contract as pii_scan_redact (rows of a conversation contiguous, in order).  Each row is
 * appended to its conversation's window and produces the redacted window text ending at that row:
 *   out_bytes/out_offsets : one redacted window per row
 *   spans                 : window findings, utt = row, start/end = byte offsets in the JOINED window
 *   win_ctx               : optional int16[n_utt], the context group the window used (-1 none): the
 *                           expected_pii_type a request right after the row would GET (an AGENT row's
 *                           own keyword hit, else the live record)
 * AGENT rows update the conversation context exactly as in pii_scan_redact (so passing a row to both
 * calls is idempotent).  On any error nothing is committed (context, window history). */
int pii_rescan_window(struct pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                      const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us,
                      uint8_t* out_bytes, uint64_t out_cap, uint64_t* out_offsets,
                      pii_span* spans, uint32_t span_cap, uint32_t* n_spans, int16_t* win_ctx);
int pii_rescan_window_device(struct pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets,
                             uint32_t n_utt, const uint32_t* d_conv_slot, const uint8_t* d_role,
                             const int64_t* d_ts_us, uint8_t* d_out_bytes, uint64_t out_cap,
                             uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap,
                             int16_t* d_win_ctx, void* stream);
/* The same with offsets[0] and the byte size stated by the caller (as pii_scan_redact_device_ex):
 * a re-scan step enqueues without any device-to-host read. */
int pii_rescan_window_device_ex(struct pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets,
                                uint32_t n_utt, uint64_t batch_base, uint64_t batch_bytes,
                                const uint32_t* d_conv_slot, const uint8_t* d_role, const int64_t* d_ts_us,
                                uint8_t* d_out_bytes, uint64_t out_cap, uint64_t* d_out_offsets,
                                pii_span* d_spans, uint32_t span_cap, int16_t* d_win_ctx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PII_ENGINE_H */
