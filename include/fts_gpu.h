/*
 * fts_gpu.h — C-ABI of the MI355X batch verifier for zkatdlog ("nogh" v1)
 * token proofs on BN254.
 *
 * This is the drop-in boundary: a Go validator binds these symbols through
 * cgo.  Only plain pointers and sizes cross it; the
 * library owns all device memory, streams and tables per context.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * token/core/zkatdlog/nogh/v1/ in murongshaozong/fabric-token-sdk):
 *   fts_ctx_create            crypto/setup.go:319-372   PublicParams.Deserialize
 *                             + driver/base.go:39-46     DefaultValidator (context build)
 *   fts_rp_verify_batch       crypto/rp/bulletproof.go:184-205,252-333
 *                                                       NewRangeVerifier + (*rangeVerifier).Verify
 *                             crypto/rp/ipa.go:190-262  (*ipaVerifier).Verify (called from it)
 *   fts_transfer_verify_batch crypto/transfer/transfer.go:49-60,153-197
 *                                                       transfer.NewVerifier + (*Verifier).Verify
 *                             (validator/validator_transfer.go:96-110 TransferZKProofValidate)
 *   fts_issue_verify_batch    crypto/issue/verifier.go:24-57 issue.NewVerifier + Verify
 *                             (validator/validator_issue.go:28-32 IssueValidate)
 *   fts_status_str            the reference's error strings (bulletproof.go:255-323,
 *                             ipa.go:193-258, rangecorrectness.go:139-159,
 *                             typeandsum.go:232-274, sametype.go:180, transfer.go:192-196)
 *   fts_*_prove               crypto/rp/bulletproof.go:209-249, transfer/transfer.go:69-150,
 *                             issue/prover.go:46-112 (host prover: synthetic inputs)
 *
 * Return values: every function returns FTS_API_OK (0) or a negative
 * FTS_API_* code for API/driver errors (bad argument, HIP failure).
 * Per-item verdicts go to caller-owned int32 arrays as fts_status values.
 * Thread safety: every verify entry point may be called concurrently.  Calls queue
 * at one dispatcher per context; a free lane (FTS_LANES, default 4: its own HIP
 * streams and workspace) takes the queue's head calls as ONE device pass -- the
 * range proofs of staged batches, transfer, issue, mixed and request calls are
 * verified together (up to FTS_COALESCE_MAX proofs), each call's sigma proofs beside
 * them -- and every call gets exactly the verdicts it would get alone.
 */
#ifndef FTS_GPU_H
#define FTS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-item verdicts (1:1 with the reference's distinct error strings) ---- */
enum fts_status {
  FTS_OK = 0,
  FTS_E_MALFORMED = 1,      /* deserialization error, or input on which the reference panics */
  FTS_E_RP_NIL = 2,         /* "invalid range proof: nil elements"   bulletproof.go:255-264 */
  FTS_E_RP_INVALID = 3,     /* "invalid range proof"                 bulletproof.go:323 */
  FTS_E_IPA_NIL = 4,        /* "invalid IPA proof: nil elements"     ipa.go:193,227 */
  FTS_E_IPA_LEN = 5,        /* "invalid IPA proof"                   ipa.go:197 */
  FTS_E_IPA_INVALID = 6,    /* "invalid IPA"                         ipa.go:258 */
  FTS_E_RC_COUNT = 7,       /* "invalid range proof" (#proofs != #commitments) rangecorrectness.go:139 */
  FTS_E_TAS_INVALID = 8,    /* "invalid sum and type proof"          typeandsum.go:232,274 */
  FTS_E_ST_INVALID = 9,     /* "invalid same type proof"             sametype.go:180 */
  FTS_E_NOT_RUN = 10,       /* item not evaluated (batch aborted by an API error) */
  FTS_E_ACTION_INVALID = 11, /* action fails its structural Validate() before the ZK proof:
                               issue/action.go:161-185,273-282; transfer/action.go:244-283 */
  FTS_E_OPEN_MISMATCH = 12, /* "output at index [%d] does not match the provided opening"
                               audit/auditor.go:236-238; "... output does not match provided
                               opening" token/token.go:78-80 */
  FTS_E_SIG_MALFORMED = 13, /* asn1.Unmarshal of the ECDSA signature failed   validator/ecdsa/ecdsa.go:84-87 */
  FTS_E_SIG_NOT_LOW_S = 14, /* "signature is not in lowS"                     validator/ecdsa/ecdsa.go:103-105 */
  FTS_E_SIG_INVALID = 15,   /* "signature not valid" (ecdsa.Verify false)     validator/ecdsa/ecdsa.go:107-110 */
  FTS_E_NYM_MALFORMED = 16, /* idemix nym signature empty / proto.Unmarshal failed (bccsp NymSigner.Verify) */
  FTS_E_NYM_BADKEY = 17,    /* nym public key import failed (idemix/crypto/deserializer.go:49-56) */
  FTS_E_NYM_INVALID = 18,   /* "pseudonym signature invalid: zero-knowledge proof is invalid"
                               (NymSignature.Ver, via idemix/crypto/id.go:151-161) */
  /* idemix identity validity (crypto/id.go:74-108 -> IBM/idemix Signature.Ver), in the order checked: */
  FTS_E_ID_MALFORMED = 19,  /* empty identity, SerializedIdemixIdentity / Signature proto or a point
                               encoding does not parse (crypto/deserializer.go:37-47) */
  FTS_E_ID_BADNYM = 20,     /* nym public key import failed (crypto/deserializer.go:49-56) */
  FTS_E_ID_NO_EIDNYM = 21,  /* "no EidNym provided but ExpectEidNym required" */
  FTS_E_ID_NO_RHNYM = 22,   /* "no RhNym provided but ExpectEidNymRhNym required" */
  FTS_E_ID_REVOCATION = 23, /* revocation algorithm other than ALG_NO_REVOCATION */
  FTS_E_ID_APRIME = 24,     /* "signature invalid: APrime = 1" */
  FTS_E_ID_PAIRING = 25,    /* "signature invalid: APrime and ABar don't have the expected structure" */
  FTS_E_ID_ZK = 26          /* "signature invalid: zero-knowledge proof is invalid" */
};

/* ---- API return codes ---- */
#define FTS_API_OK 0
#define FTS_API_EINVAL (-1)   /* bad argument / NULL pointer */
#define FTS_API_EPP (-2)      /* public parameters rejected (setup.go:319-372,444-489) */
#define FTS_API_EDEVICE (-3)  /* HIP runtime / device failure */
#define FTS_API_ENOMEM (-4)
#define FTS_API_ESIZE (-5)    /* unsupported bit length / batch shape */

/* device argument of fts_ctx_create*: host-only context (parsing + prover, no GPU) */
#define FTS_DEVICE_NONE (-2)

typedef struct fts_ctx fts_ctx;
typedef struct fts_rp_batch fts_rp_batch;

typedef struct fts_pp_info {
  uint32_t bit_length;      /* RangeProofParams.BitLength (8/16/32/64) */
  uint32_t rounds;          /* RangeProofParams.NumberOfRounds */
  uint32_t curve_id;        /* always 1 (BN254) */
  int32_t device;           /* HIP device ordinal the context runs on */
  uint64_t max_token;
  uint64_t table_bytes;     /* device bytes of fixed-base tables */
  uint32_t wide_bits;       /* window width of the per-proof bases' tables: 22 (11 additions per
                               product, 1.5 GiB per base) or 20 (12, 436 MiB); fts_ctx_opts */
  uint32_t lanes;           /* concurrent device passes (execution lanes) */
} fts_pp_info;

/* Context options (fts_ctx_create_opts); zero-initialise, then set what you need. */
typedef struct fts_ctx_opts {
  uint32_t bit_length;      /* 0: the PP's own (else as fts_ctx_create_bits) */
  int32_t wide_bits;        /* 20 or 22: force the per-proof bases' window width; 0: by budget */
  uint64_t table_budget;    /* with wide_bits 0: the most device bytes this context's fixed-base
                               tables may take -- 22-bit tables only when all of them fit (at
                               n = 64: 104 GiB; 20-bit: 33 GiB).  0: 22-bit only when the free
                               HBM at creation exceeds them + 8 GiB per lane + 128 GiB (the first
                               context on an empty MI355X), falling back to 20-bit if the
                               allocation fails.  FTS_WIDE_BITS overrides the budget. */
  int32_t lanes;            /* 0: FTS_LANES or 4 */
  int32_t reserved;
} fts_ctx_opts;

/* One transfer action: commitments as 64-byte X||Y big-endian (G1.Bytes()). */
typedef struct fts_transfer_item {
  const uint8_t* inputs;    /* n_in  * 64 bytes */
  size_t n_in;
  const uint8_t* outputs;   /* n_out * 64 bytes */
  size_t n_out;
  const uint8_t* proof;     /* transfer.Proof DER (transfer.go:29-40) */
  size_t proof_len;
} fts_transfer_item;

/* One issue action. */
typedef struct fts_issue_item {
  const uint8_t* tokens;    /* n_tok * 64 bytes */
  size_t n_tok;
  const uint8_t* proof;     /* issue.Proof DER (issue/prover.go:27-37) */
  size_t proof_len;
} fts_issue_item;

/* ---- context ---- */
/* pp: PublicParams.Serialize() bytes (JSON container {"identifier","raw"}).
 * device: HIP device ordinal (-1: current device, FTS_DEVICE_NONE: host-only). */
int fts_ctx_create(const uint8_t* pp, size_t pp_len, int device, fts_ctx** out);
/* Same generators, range proofs truncated to bit_length (Setup(bit_length) semantics,
 * setup.go:388-406: labels do not depend on the bit length). */
int fts_ctx_create_bits(const uint8_t* pp, size_t pp_len, uint32_t bit_length, int device, fts_ctx** out);
/* Same, with explicit options (table budget, window width, lanes); opts may be NULL. */
int fts_ctx_create_opts(const uint8_t* pp, size_t pp_len, int device, const fts_ctx_opts* opts, fts_ctx** out);
/* Multi-device context (SURVEY §8b device_mask; the reference verifies every action
 * independently, core/common/validator.go:215-224): one child context per device (its
 * own tables, lanes, streams).  Every batch entry point below splits the caller's batch
 * into contiguous shards balanced by cost (fts_shard_plan: range proofs per action),
 * runs the shards on their devices concurrently and returns the verdicts in the
 * caller's order; fts_msm_g1 sums the devices' partial MSM points on the host.
 * Provers, staged MSMs, timings and debug hooks use the first device.  devices[] may
 * repeat an ordinal (several shards on one device).  bit_length 0: the PP's own. */
int fts_ctx_create_devices(const uint8_t* pp, size_t pp_len, uint32_t bit_length, const int32_t* devices, int ndev,
                           fts_ctx** out);
/* bit d of device_mask = HIP device d */
int fts_ctx_create_mask(const uint8_t* pp, size_t pp_len, uint32_t bit_length, uint64_t device_mask, fts_ctx** out);
/* devices of the context (up to cap written); returns their number (0: host-only) */
int fts_ctx_devices(const fts_ctx* ctx, int32_t* devices, int cap);
/* contiguous split of n items into nshards shards of (near) equal total weight
 * (weights NULL: equal weights): shard j = [bounds[j], bounds[j+1]), bounds[0] = 0,
 * bounds[nshards] = n.  Host-only; the split every multi-device entry point uses. */
int fts_shard_plan(size_t n, const double* weights, int nshards, size_t* bounds);
void fts_ctx_destroy(fts_ctx* ctx);
int fts_ctx_info(const fts_ctx* ctx, fts_pp_info* out);

/* ---- verification (host buffers in, verdicts out) ---- */
/* n standalone range proofs: rp_der[i] = RangeProof.Serialize() (bulletproof.go:93-95),
 * com64 = n * 64-byte commitments V_i.  status[i] <- fts_status. */
int fts_rp_verify_batch(fts_ctx* ctx, size_t n, const uint8_t* const* rp_der, const size_t* rp_len,
                        const uint8_t* com64, int32_t* status);
/* status[i] <- fts_status; fail_index[i] <- index of the failing range proof (-1 if none). */
int fts_transfer_verify_batch(fts_ctx* ctx, size_t n, const fts_transfer_item* items, int32_t* status,
                              int32_t* fail_index);
int fts_issue_verify_batch(fts_ctx* ctx, size_t n, const fts_issue_item* items, int32_t* status,
                           int32_t* fail_index);

/* Transfers and issues of many token requests in ONE device pass (BASELINE config C5):
 * verdicts identical to fts_transfer_verify_batch / fts_issue_verify_batch on the same
 * items.  fail_tr / fail_is may be NULL. */
int fts_actions_verify_batch(fts_ctx* ctx, size_t n_tr, const fts_transfer_item* transfers, size_t n_is,
                             const fts_issue_item* issues, int32_t* status_tr, int32_t* fail_tr, int32_t* status_is,
                             int32_t* fail_is);

/* ---- raw TokenRequest ingest (replaces the deserialisation + ZK half of
 * Validator.VerifyTokenRequestFromRaw, core/common/validator.go:78-130) ----
 * req[i] = TokenRequest.Bytes() (driver/request.go:38-53, protos request.proto:95-100).
 * Every request is decoded on the host (TokenRequest.FromBytes, DeserializeActions:
 * validator/validator.go:27-47, the actions' Deserialize + Validate), then the ZK proofs
 * of ALL actions of ALL n requests are verified in ONE device pass.
 *   status[i]      <- FTS_OK, or the verdict of the request's first failing action in
 *                     the reference's order (every issue, then every transfer), or
 *                     FTS_E_MALFORMED when the request / an action does not deserialise
 *   fail_action[i] <- index in TokenRequest.actions of that action (-1: request level
 *                     or OK)
 *   fail_index[i]  <- index of the failing range proof inside that action (-1 if none)
 * Not evaluated here (stay with the caller's Go code): signatures, auditor signature,
 * issuer allow-list, upgrade-witness commitment, HTLC scripts, ledger lookups.
 * fail_action / fail_index may be NULL. */
int fts_request_verify_batch(fts_ctx* ctx, size_t n, const uint8_t* const* req, const size_t* req_len,
                             int32_t* status, int32_t* fail_action, int32_t* fail_index);
/* Host-only decode of one request (no device, ctx not needed): the deserialisation verdict
 * (status, fail_action as above), the action counts, and the first action (reference order)
 * whose structural check fails before its proof (pre_status FTS_E_ACTION_INVALID /
 * FTS_E_MALFORMED, pre_action its index; FTS_OK / -1 if none). */
int fts_request_inspect(const uint8_t* req, size_t req_len, int32_t* status, int32_t* fail_action,
                        int32_t* n_issue, int32_t* n_transfer, int32_t* pre_status, int32_t* pre_action);

/* ---- device-resident batches (parse + upload once, verify many times) ---- */
int fts_rp_batch_stage(fts_ctx* ctx, size_t n, const uint8_t* const* rp_der, const size_t* rp_len,
                       const uint8_t* com64, fts_rp_batch** out);
/* runs the whole GPU verification of a staged batch; status may be NULL.
 * Thread-safe: concurrent calls on DIFFERENT batches run on different lanes
 * (stream pairs, FTS_LANES env, default 4) and overlap on the device; batches
 * submitted while every lane is busy are coalesced into one device pass of
 * up to FTS_COALESCE_MAX proofs (default 81920).  Verdicts are per proof and
 * independent of the grouping. */
int fts_rp_batch_verify(fts_ctx* ctx, fts_rp_batch* b, int32_t* status);
/* pre-allocate every lane's workspace for device passes of up to max_pass_proofs
 * range proofs (0: FTS_COALESCE_MAX) so that no allocation -- and no device-wide
 * synchronisation -- happens once batches flow; call once after fts_ctx_create */
int fts_ctx_reserve(fts_ctx* ctx, size_t max_pass_proofs);
/* number of staged batches (including b) in the device pass that verified b last */
int fts_rp_batch_merged(const fts_rp_batch* b);
/* Test hook: no device pass starts until n calls (staged batches and action calls of any
 * entry point) are queued, then the queue forms passes as usual (one-shot; n = 0 releases).
 * Makes "these calls share one pass" deterministic in tests. */
int fts_debug_hold(fts_ctx* ctx, int n);
/* Host cost of an action call's staging (DER parse into the device layout, no device;
 * ctx must be host-only: FTS_DEVICE_NONE): ms_avg[0..3] <- mean wall ms over reps of the
 * whole staging and of its three steps (shapes, layout, decode). */
int fts_debug_stage_actions(fts_ctx* ctx, size_t n_tr, const fts_transfer_item* transfers, size_t n_is,
                            const fts_issue_item* issues, int reps, float* ms_avg);
/* dispatcher counters since context creation: out[0] device passes, out[1] calls served,
 * out[2] most calls in one pass, out[3] action calls (transfer / issue / actions / request) */
int fts_debug_dispatch_stats(const fts_ctx* ctx, int64_t* out);
/* per-kernel device time (ms) and algorithmic u32 MADs of b's last verification */
int fts_rp_batch_timings(const fts_rp_batch* b, const char** names, float* ms, double* mads, int cap);
void fts_rp_batch_free(fts_rp_batch* b);
/* device time of the last fts_rp_batch_verify, per kernel class (ms); returns count filled */
int fts_last_timings(const fts_ctx* ctx, const char** names, float* ms, int cap);
/* same, plus the algorithmic u32 MAD count of each launch (DESIGN.md cost model; 0 for
 * kernels without field products, e.g. SHA-256) */
int fts_last_timings_ex(const fts_ctx* ctx, const char** names, float* ms, double* mads, int cap);

/* parity/debug hook: exact intermediates of proof i of the last range-proof run
 * (ch_out: (8+2k) x 32-byte BE Fr [x, x^2, y, y^-1, z, z^2, polEval, x0, x_j..., x_j^-1...],
 *  com_out: 64-byte com, hp_out: n x 64-byte H'_i); any pointer may be NULL */
int fts_debug_rp_intermediates(fts_ctx* ctx, size_t i, uint8_t* ch_out, uint8_t* com_out, uint8_t* hp_out);

/* debug: bucket occupancy of the last RLC MSM: out[0] max bucket count, out[1] its index,
 * out[2] total buckets, out[3] non-empty buckets */
int fts_debug_msm_stats(fts_ctx* ctx, int64_t* out);

/* ---- standalone BN254 G1 multi-scalar multiplication (BASELINE config C3) ----
 * out64 <- sum_i k_i P_i as 64-byte X||Y BE (identity: 64 zero bytes), the value
 * gnark-crypto's G1 MultiExp / mathlib G1.Mul + Add return.
 * points64: n x 64-byte X||Y BE, each checked like NewG1FromBytes (asn1.go:148): flag
 * bits, canonical coordinates, on the curve; 64 zero bytes = identity.  A rejected
 * point makes the call return FTS_API_EINVAL.
 * scalars32: n x 32-byte BE integers, used mod r (G1.Mul semantics).
 * Device Pippenger MSM (GLV split, signed windows, counting-sort buckets; msm.hip). */
typedef struct fts_msm_batch fts_msm_batch;
int fts_msm_g1(fts_ctx* ctx, size_t n, const uint8_t* points64, const uint8_t* scalars32, uint8_t* out64);
/* device-resident variant: upload + validate once, run many times */
int fts_msm_stage(fts_ctx* ctx, size_t n, const uint8_t* points64, const uint8_t* scalars32, fts_msm_batch** out);
int fts_msm_run(fts_ctx* ctx, fts_msm_batch* b, uint8_t* out64);
/* config C3 at scale (points k_i G with uniform k_i): n DISTINCT points
 * P_i = k_i * ped1 (the PP's ped[1], a generator of G1) computed on the device from the
 * context's fixed-base table, k32 / scalars32: n x 32-byte BE integers used mod r.  The
 * result of fts_msm_run is then (sum_i s_i k_i mod r) * ped1 (closed form for tests). */
int fts_msm_stage_multiples(fts_ctx* ctx, size_t n, const uint8_t* k32, const uint8_t* scalars32, fts_msm_batch** out);
/* the staged points [lo, lo + count) of b as 64-byte X||Y BE (identity = 64 zero bytes):
 * the C3 CPU baseline runs its Pippenger over the same distinct points */
int fts_msm_points(fts_ctx* ctx, const fts_msm_batch* b, size_t lo, size_t count, uint8_t* out64);
/* per-kernel device time (ms) and algorithmic u32 MADs of b's last run */
int fts_msm_timings(const fts_msm_batch* b, const char** names, float* ms, double* mads, int cap);
void fts_msm_free(fts_msm_batch* b);

/* ---- token opening checks (auditor / wallet) ----
 * Replaces the per-token commit() + Equals of Auditor.InspectOutput
 * (crypto/audit/auditor.go:226-238, reached from CheckIssueRequests / CheckTransferRequests
 * :178-210) and of Token.ToClear (crypto/token/token.go:69-83):
 *   status[i] <- FTS_OK iff HashToZr(type_i)*ped0 + value_i*ped1 + bf_i*ped2 == com_i
 *                FTS_E_OPEN_MISMATCH otherwise
 * com64:   token.Data as 64 B X||Y BE (G1.Bytes()), checked like NewG1FromBytes (flag bits,
 *          canonical coordinates, on the curve; 64 zero bytes = identity) -> FTS_E_MALFORMED
 * type:    metadata.Type bytes (HashToZr = SHA-256 mod r)
 * value32, bf32: Zr.Bytes() 32 B BE, used mod r (G1.Mul semantics)
 * A NULL com64 / value32 / bf32 -> FTS_E_MALFORMED (the reference returns "invalid output at
 * index [%d]" / "cannot commit a nil element", or panics on a nil Zr in the auditor's commit).
 * One device pass: three fixed-base products per token (audit_kernels.hip). */
typedef struct {
  const uint8_t* com64;
  const uint8_t* type;
  size_t type_len;
  const uint8_t* value32;
  const uint8_t* bf32;
} fts_token_opening;
int fts_token_open_batch(fts_ctx* ctx, size_t n, const fts_token_opening* items, int32_t* status);
/* The same check from the serialized form the auditor receives: meta[i] = driver.Metadata
 * bytes of output i (ASN.1 TypedToken{2, proto TokenMetadata}), decoded as
 * token.Metadata.Deserialize does (crypto/token/token.go:136-158; audit/auditor.go:296-300,
 * :370-374 call it), com64 = n x 64 B token.Data.  A metadata that does not decode, or
 * carries a nil value / blinding factor -> FTS_E_MALFORMED. */
int fts_token_metadata_open_batch(fts_ctx* ctx, size_t n, const uint8_t* com64, const uint8_t* const* meta,
                                  const size_t* meta_len, int32_t* status);
/* Host-only decode of one driver.Metadata (no device): status FTS_OK / FTS_E_MALFORMED, the
 * type as (offset, length) into meta, value / bf mod r as 32 B BE, has bit 0 / bit 1 = value /
 * bf present (non-nil). */
int fts_token_metadata_decode(const uint8_t* meta, size_t meta_len, int32_t* status, size_t* type_off,
                              size_t* type_len, uint8_t* value32, uint8_t* bf32, int32_t* has);

/* ---- error strings ---- */
const char* fts_status_str(int32_t status);

/* ---- host prover (reference prover semantics) ----
 * seed selects the prover randomness of every fts_*_prove* entry point:
 *   FTS_SEED_OS_RANDOM  secure: ChaCha20 keystreams under a fresh 256-bit getrandom() key
 *                       per call, one per proof / action (the role of crypto/rand in
 *                       Curve.NewRandomZr, rp/bulletproof.go:336-466).  Use this for real tokens.
 *   any other value     deterministic, FOR TESTS AND BENCHMARKS ONLY: item i draws from
 *                       xoshiro256**(seed + i).  Two calls whose seed ranges overlap reuse
 *                       nonces across different witnesses, which reveals the committed
 *                       values and blinding factors. */
#define FTS_SEED_OS_RANDOM UINT64_MAX
/* value < 2^bit_length expected (larger values produce a proof that fails, as in the
 * reference).  bf32: blinding factor (BE, reduced mod r).  seed: deterministic RNG seed.
 * out_der: caller buffer of out_cap bytes; *out_len <- bytes written. com64_out: V. */
int fts_rp_prove(const fts_ctx* ctx, uint64_t value, const uint8_t* bf32, uint64_t seed, uint8_t* out_der,
                 size_t out_cap, size_t* out_len, uint8_t* com64_out);
/* batch helper: n proofs with values[i], blinding factors bfs[i*32], seeds seed+i,
 * written into one buffer (offsets[i], lens[i]); uses `threads` host threads */
int fts_rp_prove_batch(const fts_ctx* ctx, size_t n, const uint64_t* values, const uint8_t* bfs, uint64_t seed,
                       int threads, uint8_t* out, size_t out_cap, size_t* offsets, size_t* lens,
                       uint8_t* com64_out);
/* Batched range-proof prover on the device: rangeProver.Prove
 * (rp/bulletproof.go:209-249, preprocess :336-466, IPA prover ipa.go:158-186,267-322) for n
 * proofs in device passes of up to 16,384 (prove_kernels.hip).  Same arguments and output as
 * fts_rp_prove_batch -- byte-identical proofs for the same seed (proof i uses seed + i; the
 * host draws the randomness, the device computes every group element, transcript and
 * Fiat-Shamir challenge).  Needs a device context. */
int fts_rp_prove_batch_gpu(fts_ctx* ctx, size_t n, const uint64_t* values, const uint8_t* bfs, uint64_t seed,
                           uint8_t* out, size_t out_cap, size_t* offsets, size_t* lens, uint8_t* com64_out);
/* Whole transfer / issue proofs on the device: the TypeAndSum
 * (transfer/typeandsum.go:189-227,280-356) or SameType (issue/sametype.go:103-149) sigma
 * proof in one kernel (thread per action), then the range proofs of every output of every
 * action in one fts_rp_prove_batch_gpu-style pass.  Action i is seeded with seed + i and the
 * output is byte-identical to fts_transfer_prove / fts_issue_prove.  Issues ignore n_in /
 * in_values / in_bfs (their tokens are the outputs). */
typedef struct {
  const uint8_t* type;
  size_t type_len;
  size_t n_in;
  const uint64_t* in_values;
  const uint8_t* in_bfs;  /* n_in x 32 B BE */
  size_t n_out;
  const uint64_t* out_values;
  const uint8_t* out_bfs; /* n_out x 32 B BE */
} fts_action_witness;
int fts_transfer_prove_batch_gpu(fts_ctx* ctx, size_t n, const fts_action_witness* w, uint64_t seed, uint8_t* out,
                                 size_t out_cap, size_t* offsets, size_t* lens);
int fts_issue_prove_batch_gpu(fts_ctx* ctx, size_t n, const fts_action_witness* w, uint64_t seed, uint8_t* out,
                              size_t out_cap, size_t* offsets, size_t* lens);
/* Token commitments (token.go:208-217): tok = H(type)*ped0 + value*ped1 + bf*ped2 */
int fts_token_commit(const fts_ctx* ctx, const uint8_t* type, size_t type_len, uint64_t value,
                     const uint8_t* bf32, uint8_t* com64_out);
/* transfer.NewProver(...).Prove(): n_in inputs / n_out outputs with witnesses */
int fts_transfer_prove(const fts_ctx* ctx, const uint8_t* type, size_t type_len, size_t n_in,
                       const uint64_t* in_values, const uint8_t* in_bfs, size_t n_out, const uint64_t* out_values,
                       const uint8_t* out_bfs, uint64_t seed, uint8_t* out_der, size_t out_cap, size_t* out_len);
/* issue.NewProver(...).Prove() */
int fts_issue_prove(const fts_ctx* ctx, const uint8_t* type, size_t type_len, size_t n_tok, const uint64_t* values,
                    const uint8_t* bfs, uint64_t seed, uint8_t* out_der, size_t out_cap, size_t* out_len);

/* ---- ECDSA P-256 owner signatures (x509 identities) ----
 * Replaces, per item, ecdsa.Verifier.Verify(message, sigma)
 * (validator/ecdsa/ecdsa.go:82-113; identical logic in
 * services/identity/x509/crypto/ecdsa.go:46-77), called by
 * TransferSignatureValidate (validator/validator_transfer.go:29-62) once per
 * input owner.  Independent of the zkatdlog public parameters: takes a device
 * ordinal, not an fts_ctx. */
typedef struct {
  const uint8_t* msg;  /* signed message; SHA-256 is computed on the device */
  size_t msg_len;
  const uint8_t* sig;  /* DER ECDSA-Sig-Value SEQUENCE{INTEGER r, INTEGER s} */
  size_t sig_len;
  const uint8_t* pk64; /* public key X||Y, 32 B big-endian each (see fts_p256_pubkey_from_pkix) */
} fts_ecdsa_item;
/* status[i] <- FTS_OK | FTS_E_SIG_MALFORMED | FTS_E_SIG_NOT_LOW_S | FTS_E_SIG_INVALID
 * (an off-curve / non-canonical public key is FTS_E_SIG_INVALID, as in Go's ecdsa.Verify). */
int fts_ecdsa_verify_batch(int device, size_t n, const fts_ecdsa_item* items, int32_t* status);
/* Host-only: the asn1.Unmarshal + IsLowS + range part of Verify; r32/s32 <- 32 B big-endian
 * (valid when *status == FTS_OK). */
int fts_ecdsa_sig_parse(const uint8_t* sig, size_t sig_len, uint8_t* r32, uint8_t* s32, int32_t* status);
/* Host-only: DER SubjectPublicKeyInfo of a P-256 key (x509.MarshalPKIXPublicKey, the body of
 * the PEM "PUBLIC KEY" block of ecdsa.Verifier.Serialize, ecdsa.go:115-150) -> X||Y.
 * FTS_API_EINVAL for anything else. */
int fts_p256_pubkey_from_pkix(const uint8_t* der, size_t len, uint8_t* pk64);
/* HIP-event durations (ms) of the last fts_ecdsa_verify_batch on `device`:
 * ms2[0] = k_ecdsa_digest, ms2[1] = k_ecdsa_verify. */
int fts_ecdsa_last_timings(int device, float* ms2);

/* ---- idemix pseudonym signatures (idemix owner identities, BN254 issuer keys) ----
 * Replaces, per item, crypto.NymSignatureVerifier.Verify(message, sigma)
 * (services/identity/idemix/crypto/id.go:145-161 -> IBM/idemix NymSignature.Ver),
 * the owner verifier that services/identity/idemix/deserializer.go:82-105 returns
 * for an idemix identity; called by TransferSignatureValidate
 * (validator/validator_transfer.go:29-62) once per input owner.
 * One handle per issuer public key (the idemix IssuerPublicKey proto, as held in
 * PublicParams.IdemixIssuerPublicKeys): HSk / HRand fixed-base tables in HBM
 * (BN254: 2 x 32 MiB; FP256BN_AMCL: 2 x 64 MiB).  FTS_API_EPP for a key that does not
 * parse or whose HSk / HRand are not on the curve. */
typedef struct fts_idemix_ipk fts_idemix_ipk;
/* curve_id: mathlib CurveID of the key (PublicParams.IdemixIssuerPublicKeys[i].Curve) */
#define FTS_CURVE_FP256BN_AMCL 0
#define FTS_CURVE_BN254 1
int fts_idemix_ipk_create(int device, const uint8_t* ipk, size_t ipk_len, int curve_id, fts_idemix_ipk** out);
void fts_idemix_ipk_destroy(fts_idemix_ipk* ipk);
typedef struct {
  const uint8_t* nym; /* NymPublicKey bytes: G1.Bytes() (BN254: 64 B raw X||Y; FP256BN: 65 B 0x04||X||Y),
                         see fts_idemix_identity_nym */
  size_t nym_len;
  const uint8_t* sig; /* NymSignature proto (proof_c, proof_s_sk, proof_s_r_nym, nonce) */
  size_t sig_len;
  const uint8_t* msg; /* signed message; hashed on the device */
  size_t msg_len;
} fts_nym_item;
/* status[i] <- FTS_OK | FTS_E_NYM_MALFORMED | FTS_E_NYM_BADKEY | FTS_E_NYM_INVALID */
int fts_nym_verify_batch(fts_idemix_ipk* ipk, size_t n, const fts_nym_item* items, int32_t* status);
/* Host-only: SerializedIdemixIdentity.nym_public_key (idemix/crypto/protos/idemix_config.proto,
 * crypto/deserializer.go:41-56); *nym points into `id`. FTS_API_EINVAL if absent or malformed. */
int fts_idemix_identity_nym(const uint8_t* id, size_t len, const uint8_t** nym, size_t* nym_len);
/* HIP-event duration (ms) of k_nym_verify in the last finished fts_nym_verify_batch on `ipk`. */
int fts_nym_last_timings(fts_idemix_ipk* ipk, float* ms);

/* ---- idemix identity validity (idemix half) ----
 * Replaces the validity check of idemix Deserializer.Deserialize(raw, true)
 * (services/identity/idemix/deserializer.go:82-93 -> crypto/deserializer.go:36-86 ->
 * crypto/id.go:74-108 verifyProof -> IBM/idemix Signature.Ver with ExpectEidNymRhNym),
 * which TransferSignatureValidate reaches for every input through
 * GetOwnerVerifier (validator/validator_transfer.go:46, core/common/deserializer.go:63-64).
 * One handle per issuer public key: fixed-base tables of HSk, HRand, HAttrs[0..3] and
 * g1 (BN254: 7 x 32 MiB; FP256BN_AMCL: 7 x 64 MiB) and the Miller-loop lines of W and g2.
 * FTS_API_EPP for a key that does not parse, lacks four attributes, or has a point off
 * its curve. */
typedef struct fts_idemix_idv fts_idemix_idv;
int fts_idemix_idv_create(int device, const uint8_t* ipk, size_t ipk_len, int curve_id, fts_idemix_idv** out);
void fts_idemix_idv_destroy(fts_idemix_idv* idv);
/* ids[i] = a serialized idemix owner identity (SerializedIdemixIdentity proto, the token's
 * Owner); status[i] <- FTS_OK or FTS_E_ID_* (the first failing check).  Thread-safe: up to
 * 8 calls on one handle run concurrently (one device slot each); more callers wait for a
 * slot.  The pairing equation is checked per group of 256 identities as one randomised
 * product (fresh getrandom weights per call, soundness 2^-128); the identities of a
 * failing group are paired one by one, so status[i] is the per-identity verdict. */
int fts_idemix_identity_verify_batch(fts_idemix_idv* idv, size_t n, const uint8_t* const* ids, const size_t* id_len,
                                     int32_t* status);
/* HIP-event durations (ms) of the last batch: [0] decode + t-values + transcript, [1] pairings
 * (the batch check and the one-by-one pairings of the identities of failing groups). */
int fts_idemix_identity_last_timings(fts_idemix_idv* idv, float* ms);
/* The last batch's pairing check: out[0] = groups of 256 identities checked with one
 * randomised pairing product each (0 with FTS_IDV_BATCH=0), out[1] = identities paired one
 * by one (those of the groups whose product was not 1; every identity with the batch off). */
int fts_idemix_identity_last_stats(fts_idemix_idv* idv, uint32_t* out);
/* Debug (tests): e(Q, P) for Q = W (which 0) or g2 (1) and P = 64 raw BE bytes (BN254),
 * after the final exponentiation (final_exp != 0) or the Miller value; out192 = 6 Fp2
 * coefficients of w^0..w^5, Montgomery, little-endian limbs. */
int fts_idemix_pairing_debug(fts_idemix_idv* idv, int which, const uint8_t* p64, int final_exp, uint32_t* out192);

#ifdef __cplusplus
}
#endif
#endif /* FTS_GPU_H */
