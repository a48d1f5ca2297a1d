/*
 * bdls_hip.h -- C ABI of libbdlship.so, the MI355X (gfx950) batched ECDSA
 * verification engine for the BDLS / Fabric signature-verification hot path.
 *
 * Drop-in boundary: the reference verifies every signature through the BCCSP
 * provider interface, one call at a time:
 *   bccsp/bccsp.go:125             BCCSP.Verify(k Key, signature, digest []byte, opts) (bool, error)
 *   bccsp/sw/impl.go:247-270       sw CSP.Verify (arg checks + verifier dispatch)
 *   bccsp/sw/ecdsa.go:41-57        verifyECDSA (DER unmarshal, low-S, crypto/ecdsa.Verify)
 *   bccsp/sw/hash.go:29-33         hasher.Hash (SHA-256)
 *   msp/identities.go:170-199      identity.Verify = Hash(msg) + Verify(pk, sig, digest)
 * The entry points below are what a `bccsp/hip` provider binds over cgo (see
 * INTEGRATION.md): plain pointers and sizes, no Go or torch types.
 *
 * Result encoding for every verify entry point:
 *   bitmap : ceil(n/8) bytes (host API) or ceil(n/64) uint64 words (device
 *            API), LSB-first: bit i set <=> record i verified (Go returns true).
 *   reason : n bytes, BH_R_* below. Codes 1..6 correspond to Go returning
 *            (false, err) from BCCSP.Verify; 7..10 to (false, nil).
 * Function return: BH_OK (0) or a negative BH_E_* (then bh_last_error()).
 * Thread-safety: all entry points may be called concurrently from several
 * host threads; calls on one device are serialized internally.
 */
#ifndef BDLS_HIP_H
#define BDLS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---- */
#define BH_OK 0
#define BH_E_INVALID (-1) /* bad argument */
#define BH_E_NOT_INIT (-2) /* bh_init not called / device not initialised */
#define BH_E_DEVICE (-3)   /* HIP runtime error */
#define BH_E_NODEV (-4)    /* no usable gfx950 device */
#define BH_E_NOMEM (-5)    /* device allocation failed */

/* ---- per-record reason codes (bit 0 of the bitmap is 1 iff BH_R_OK) ---- */
#define BH_R_OK 0
#define BH_R_EMPTY_SIG 1    /* impl.go:252  "Invalid signature. Cannot be empty."      -> error */
#define BH_R_EMPTY_DIGEST 2 /* impl.go:255  "Invalid digest. Cannot be empty."         -> error */
#define BH_R_DER 3          /* utils/ecdsa.go:44 asn1.Unmarshal failed                  -> error */
#define BH_R_R_NONPOS 4     /* utils/ecdsa.go:57 "R must be larger than zero"           -> error */
#define BH_R_S_NONPOS 5     /* utils/ecdsa.go:60 "S must be larger than zero"           -> error */
#define BH_R_HIGH_S 6       /* sw/ecdsa.go:53 "Invalid S. Must be smaller than half..." -> error */
#define BH_R_BAD_KEY 7      /* ecdsa.Verify: Q not a valid curve point                  -> false */
#define BH_R_R_RANGE 8      /* ecdsa.Verify: r >= n                                     -> false */
#define BH_R_MATH 9         /* ecdsa.Verify: x(u1 G + u2 Q) mod n != r, or infinity    -> false */
#define BH_R_S_RANGE 10     /* ecdsa.Verify: s >= n (only with BH_F_NO_LOW_S)           -> false */
#define BH_R_UNSUPPORTED 11 /* bh_verify_x509: not an ecdsa-with-SHA256 P-256 certificate
                               signature this engine checks (the caller uses Go's x509)   */

/* ---- flags ---- */
#define BH_F_HASH_SHA256 1u /* msg[i] is a message; digest = SHA-256(msg[i]) (identity.Verify) */
#define BH_F_NO_LOW_S 2u    /* do not apply Fabric's low-S rule (plain crypto/ecdsa.Verify) */
#define BH_F_KEEP_KEYS 4u   /* keys used >= 2 times in the batch get a table in the device's
                               key registry (kept across calls, see bh_keys_register) */
#define BH_F_HASH_SHA3_256 8u /* msg[i] is a message; digest = SHA3-256(msg[i]): identity.Verify
                                 of an MSP with SignatureHashFamily SHA3 (msp/identities.go:
                                 219-227, bccsp/sw/new.go:72). Exclusive with BH_F_HASH_SHA256. */
#define BH_F_ANY_LANE 16u   /* bh_verify_dev on the library's streams (stream NULL, no timing):
                               consecutive calls rotate over the device's compute lanes
                               (BH_LANES, default 3, at most 4), each with its own workspace,
                               so a pass runs beside the previous calls' passes as host
                               batches do. The k-th BH_F_ANY_LANE pass of a device is
                               ordered after the (k-4)-th (whatever lane each took and
                               whatever other work ran between them), so a caller that
                               rotates 4 output sets never has two in-flight passes
                               writing one set; bh_sync waits for every lane.
                               Ignored elsewhere (host batches already alternate lanes). */

#define BH_CURVE_P256 0
#define BH_CURVE_SECP256K1 1

/* One batch of verify records (structure of arrays). Host pointers for
 * bh_verify(), device pointers for bh_verify_dev(). */
typedef struct bh_batch {
  const uint8_t *pub;      /* n * 64 bytes: Q.x || Q.y, 32-byte big-endian each        */
  const uint8_t *sig;      /* concatenated ASN.1 DER signatures                          */
  const uint64_t *sig_off; /* n byte offsets into sig                                    */
  const uint32_t *sig_len; /* n lengths (0 -> BH_R_EMPTY_SIG)                            */
  const uint8_t *msg;      /* concatenated messages (BH_F_HASH_SHA256) or digests        */
  const uint64_t *msg_off; /* n byte offsets into msg                                    */
  const uint32_t *msg_len; /* n lengths (digest mode: 0 -> BH_R_EMPTY_DIGEST)            */
} bh_batch;

/* The same records in the COMPACT host layout (round 4; VERDICT r3: the host
 * path sat at its PCIe bound with 24 B of u64 offsets + u32 lengths per
 * record and a 64-byte key copy per record). A Go BatchVerify holds bccsp.Key
 * objects, many of them the same identity's key (the MSP identity cache), so
 * the binding passes each distinct key once and a u32 index per record;
 * offsets are the prefix sums of the lengths (the device computes them), and
 * a batch of equal-length messages (digests, fixed-size payloads) sends no
 * lengths at all. 339 B per config-2 record instead of 424. Verification is
 * bit-for-bit that of the expanded bh_batch, record i having key keys[key_idx[i]],
 * signature and message the i-th spans of sig / msg. Host pointers. */
typedef struct bh_cbatch {
  const uint8_t *keys;      /* nkeys * 64: distinct public keys X || Y            */
  const uint32_t *key_idx;  /* n: record i's key index (< nkeys); NULL: keys holds
                               one key per record, in record order (nkeys = n)   */
  size_t nkeys;
  const uint8_t *sig;       /* concatenated DER signatures, record order         */
  const uint32_t *sig_len;  /* n lengths; record i's offset = sum of the earlier  */
  const uint8_t *msg;       /* concatenated messages (BH_F_HASH_*) or digests     */
  const uint32_t *msg_len;  /* n lengths, or NULL: every message is msg_stride B  */
  uint32_t msg_stride;
} bh_cbatch;

/* Per-call stage timing (milliseconds, HIP events on the launch stream) and
 * routing counts. */
typedef struct bh_timing {
  float prep_ms;       /* parse + checks + SHA-256 / BLAKE2b + Montgomery inputs */
  float inv_ms;        /* batched s^-1 mod n, u1, u2 */
  float plan_ms;       /* registry lookup + public-key dedup + routing */
  float build_ladder_ms; /* one grid: per-key fixed-base table builds and the
                            variable-base ladder for records without a table */
  float publish_ms;    /* registry publication of new tables (BH_F_KEEP_KEYS) */
  float keycomb_ms;    /* u2 Q from key tables + u1 G + x check, bitmap */
  uint32_t n_keycomb;  /* records verified on the key-table path */
  uint32_t n_ladder;   /* records verified on the ladder path */
  uint32_t n_keytables; /* tables built in this call */
  uint32_t wide;       /* lanes per record on the key-table path */
} bh_timing;

/* Initialise the devices in device_mask (bit d = HIP device d; 0 = all
 * visible). Builds the per-device fixed-base tables. Idempotent. */
int bh_init(uint32_t device_mask, uint32_t flags);
int bh_shutdown(void);
int bh_device_count(void);          /* devices initialised by bh_init */
const char *bh_last_error(void);    /* thread-local message for the last failure */
const char *bh_version(void);

/* Device-memory bytes of library workspace needed per device for n records. */
size_t bh_workspace_bytes(size_t n);

/* Host-memory batch: copies to the devices, shards [0,n) over all initialised
 * devices (contiguous ranges, no collective), gathers bitmap and reasons.
 * curve: BH_CURVE_P256 (the Fabric/BCCSP path; secp256k1 BDLS messages use
 * bh_verify_bdls). */
int bh_verify(int curve, const bh_batch *b, size_t n, uint32_t flags, uint8_t *bitmap,
              uint8_t *reason);

/* bh_verify with two-span messages: record i's signed bytes are
 * msg[msg_off[i], +msg_len[i]) || msg[msg2_off[i], +msg2_len[i]) (msg2_len 0 =
 * one span), hashed on the device (BH_F_HASH_SHA256 or BH_F_HASH_SHA3_256
 * required). Replaces the host-side concatenation of a Fabric endorsement's
 * SignedData, Data = prp || endorser (core/common/validation/statebased/
 * validator_keylevel.go:246-260; core/committer/txvalidator/v20/plugindispatcher),
 * so both spans can point into the serialized block itself. */
int bh_verify_2seg(int curve, const bh_batch *b, const uint64_t *msg2_off,
                   const uint32_t *msg2_len, size_t n, uint32_t flags, uint8_t *bitmap,
                   uint8_t *reason);

/* Asynchronous form of bh_verify (the pipelined BatchVerify): enqueues the
 * upload (copy stream), the verify passes and the result download (compute
 * stream) on every device and returns at once with *job. bh_verify_wait(job)
 * blocks until the batch is done, writes bitmap / reason and frees the job;
 * every submitted job must be waited exactly once. The caller's input
 * buffers must stay valid and unchanged until then. With two jobs in flight
 * per device, the next batch's H2D runs under this batch's kernels; this needs
 * page-locked inputs (bh_host_alloc) -- pageable inputs are correct but their
 * upload is staged synchronously by the HIP runtime. bh_verify = submit+wait. */
typedef struct bh_job bh_job;
int bh_verify_submit(int curve, const bh_batch *b, size_t n, uint32_t flags, uint8_t *bitmap,
                     uint8_t *reason, bh_job **job);
int bh_verify_wait(bh_job *job);

/* Page-locked host memory, DMA-able by every device (hipHostMalloc portable).
 * A cgo caller packs its SoA batch straight into it (no further copy). */
int bh_host_alloc(size_t bytes, void **ptr);
int bh_host_free(void *ptr);

/* Device-resident batch on one device: every pointer in *b and the outputs
 * are device pointers on `device`. Enqueued on `stream` (hipStream_t; NULL =
 * the library's stream for that device) and synchronised before return when
 * timing != NULL (then filled) or when sync != 0. bitmap_words: ceil(n/64)
 * uint64 words. */
int bh_verify_dev(int device, int curve, const bh_batch *b, size_t n, uint32_t flags,
                  uint64_t *bitmap_words, uint8_t *reason, void *stream, int sync,
                  bh_timing *timing);

/* Single signature with exact BCCSP.Verify semantics (the sw provider's
 * Verify for an ECDSA P-256 public key, bccsp/sw/impl.go:247-270). *valid =
 * 1/0, *reason = BH_R_*; return BH_OK unless the engine itself failed.
 * Concurrent callers are COALESCED (the drop-in Verify is called by up to
 * validatorPoolSize goroutines at once, core/peer/config.go:269-272): each
 * call joins the batch being filled and blocks; a library thread submits that
 * batch as soon as a pipeline slot is free (a lone call goes at once; under
 * load, calls arriving while one batch runs share the next device pass).
 * BH_COALESCE_US (environment, default 0) makes an idle flusher linger that
 * many microseconds for more calls. The caller's buffers are copied before
 * the call blocks. */
int bh_csp_verify_p256(const uint8_t pub[64], const uint8_t *sig, size_t sig_len,
                       const uint8_t *digest, size_t digest_len, int *valid, int *reason);
/* Coalescer counters: out[0] single calls served, out[1] device batches they
 * formed, out[2] largest batch. */
int bh_csp_stats(uint64_t out[3]);

/* bh_verify / bh_verify_submit on a compact batch (see bh_cbatch): same
 * results, flags and curves (BH_CURVE_P256), same pipeline and job handles
 * (collect with bh_verify_wait). Replaces the same reference interfaces as
 * bh_verify: BatchVerify over bccsp/sw/impl.go:247-270 / msp identities.go:
 * 170-199. BH_E_INVALID for a key index >= nkeys or a null required field. */
int bh_verify_compact(int curve, const bh_cbatch *b, size_t n, uint32_t flags, uint8_t *bitmap,
                      uint8_t *reason);
int bh_verify_compact_submit(int curve, const bh_cbatch *b, size_t n, uint32_t flags,
                             uint8_t *bitmap, uint8_t *reason, bh_job **job);

/* ---- Staged BatchVerify (round 6) ------------------------------------------
 * BatchVerify straight from the caller's own (pageable, per-record) buffers:
 * the library packs each shard into page-locked staging it owns and reuses
 * (pipeline slot buffers), on a pool of worker threads -- key de-duplication
 * by a lock-free hash table (each distinct key uploaded once + a u32 index per
 * record, the compact layout), lengths, and the signature and message bytes
 * in one pass per record, in chunks whose H2D copies start while the next
 * chunk is packed (include/../bdls_amd/csrc/pack.h).
 * Replaces the per-call packing a Go BatchVerify did on one goroutine into a
 * fresh bh_host_alloc (INTEGRATION.md 2 packBatch) -- the batch points
 * common/policies/policy.go:363-395 and core/committer/txvalidator/v20/
 * validator.go:193-208 -- and the per-call bh_host_alloc/free. Results,
 * flags, curve (BH_CURVE_P256) and job handles as bh_verify_submit (collect
 * with bh_verify_wait); the caller's buffers must stay valid until the
 * submit call RETURNS (everything is copied by then), not until the wait.
 * Worker threads: BH_PACK_THREADS, default the CPUs the process may use
 * (affinity, cgroup quota) less one, at most 15. */
int bh_batch_verify(int curve, const bh_batch *b, size_t n, uint32_t flags, uint8_t *bitmap,
                    uint8_t *reason);
int bh_batch_verify_submit(int curve, const bh_batch *b, size_t n, uint32_t flags,
                           uint8_t *bitmap, uint8_t *reason, bh_job **job);
/* The same records as separate caller buffers -- the form a cgo binding
 * hands over without flattening in Go (pointers pinned with runtime.Pinner,
 * Go >= 1.21): per record its 64-byte key X || Y, its DER signature and its
 * message (BH_F_HASH_*) or digest. A NULL signature / message pointer is a
 * zero-length field (Go's nil slice: BH_R_EMPTY_SIG / BH_R_EMPTY_DIGEST or the
 * hash of the empty message); a NULL key pointer reads as the all-zero point
 * (BH_R_BAD_KEY). Records sharing a key may pass the same pointer or equal
 * bytes: the library de-duplicates by content. */
typedef struct bh_pbatch {
  const uint8_t *const *pub;  /* n pointers to 64 bytes Q.x || Q.y                 */
  const uint8_t *const *sig;  /* n pointers to DER signatures                     */
  const uint32_t *sig_len;
  const uint8_t *const *msg;  /* n pointers to messages (BH_F_HASH_*) or digests  */
  const uint32_t *msg_len;
} bh_pbatch;
int bh_batch_verify_ptrs(int curve, const bh_pbatch *b, size_t n, uint32_t flags,
                         uint8_t *bitmap, uint8_t *reason);
int bh_batch_verify_ptrs_submit(int curve, const bh_pbatch *b, size_t n, uint32_t flags,
                                uint8_t *bitmap, uint8_t *reason, bh_job **job);
/* The last staged shard's packing: out[0] plan ms (lengths -> byte offsets),
 * [1] fill ms (lengths, keys + indices, bytes; the chunks' H2D copies queued
 * as they complete), [2] worker threads,
 * [3] chunks, [4] keys de-duplicated (1/0), [5] keys uploaded, [6] records,
 * [7] the sample's distinct-key estimate (0: no repeat seen), [8] table
 * rebuilds, [9] staged shards since start. Not in the reference
 * (operations metrics). */
int bh_pack_stats(double out[10]);

/* Device batches since bh_init over every entry point: out[0] batches launched
 * (one per device pass sequence of a call or shard, one per latency-path
 * batch), out[1] records they carried. Lets a consumer prove it issued no
 * device work (a phase-2 policy evaluation whose signatures
 * phase 1 already verified). Not in the reference: an observability hook. */
int bh_device_stats(uint64_t out[2]);

/* Host-side Go-exact DER unmarshal (bccsp/utils/ecdsa.go:41-65). Returns the
 * reason (BH_R_OK, BH_R_DER, BH_R_R_NONPOS, BH_R_S_NONPOS); on BH_R_OK fills
 * r, s (32-byte big-endian) or sets *r_big / *s_big when a value exceeds 256
 * bits. Pure host code, no device needed. */
int bh_parse_der_sig(const uint8_t *der, size_t len, uint8_t r[32], uint8_t s[32], int *r_big,
                     int *s_big);

/* ---- BDLS consensus messages -------------------------------------------
 * One record = one vendor/github.com/BDLS-bft/bdls/message.go SignedProto.
 * Verification restates SignedProto.Verify (message.go:170-184): hash =
 * SignedProto.Hash() (BLAKE2b-256 over "BDLS_CONSENSUS_SIGNATURE" || Version
 * u32-LE || X || Y || len(Message) u32-LE || Message, message.go:97-138), then
 * Go crypto/ecdsa.Verify with R, S = big.Int.SetBytes(R), SetBytes(S).
 * curve BH_CURVE_SECP256K1: as wired in orderer/consensus/bdls/chain.go:60-61
 * (Go verifyLegacy); BH_CURVE_P256: the curve-generic BDLS library with P-256
 * keys (verifyNISTEC). No low-S rule. Result reasons: BH_R_OK or a reject
 * code (every reject is Verify() == false). Off-curve keys are rejected with
 * BH_R_BAD_KEY on both curves (BDLS only admits registered participants'
 * keys, consensus.go:456-466). */
typedef struct bh_bdls_batch {
  const uint8_t *xy;       /* n * 64: SignedProto.X || SignedProto.Y (32 B each)    */
  const uint8_t *r;        /* concatenated SignedProto.R (big-endian, any length)   */
  const uint64_t *r_off;
  const uint32_t *r_len;
  const uint8_t *s;        /* concatenated SignedProto.S                            */
  const uint64_t *s_off;
  const uint32_t *s_len;
  const uint32_t *version; /* SignedProto.Version                                   */
  const uint8_t *msg;      /* concatenated SignedProto.Message                      */
  const uint64_t *msg_off;
  const uint32_t *msg_len;
} bh_bdls_batch;

/* Host buffers, first initialised device (BDLS rounds are hundreds of records). */
int bh_verify_bdls(int curve, const bh_bdls_batch *b, size_t n, uint8_t *bitmap,
                   uint8_t *reason);
/* Device-resident; semantics of bh_verify_dev. */
int bh_verify_bdls_dev(int device, int curve, const bh_bdls_batch *b, size_t n,
                       uint64_t *bitmap_words, uint8_t *reason, void *stream, int sync,
                       bh_timing *timing);

/* ---- BDLS drained-batch pre-verification ------------------------------------
 * Replaces the per-message signature work of agent-tcp/tcp_peer.go:176-192
 * (inputConsensusMessage drains the queued raw messages and calls
 * Consensus.ReceiveMessage one by one) with ONE device batch: every
 * SignedProto reachable from the drained messages -- the outer one, each
 * Message.Proof of a <lock>/<select>/<decide>, Message.LockRelease and the
 * proofs of the <lock> it embeds, and (recursively, depth <= 8) the proofs a
 * <resync> pushes to the loopback -- is decoded (gogo/protobuf wire format,
 * message.pb.go Unmarshal semantics), gated on the participant set
 * (consensus.go:449-470) and verified with SignedProto.Verify semantics.
 *
 * results[i].status is the first failure among the checks that depend only on
 * the message bytes and the participant list, in the order Go runs them
 * (receiveMessage :1209-1226, verifyMessage :449-493, verifyLockMessage
 * :520-600, verifySelectMessage :628-728, verifyDecideMessage :829-902,
 * verifyLockReleaseMessage :604-623). Checks that need consensus state or
 * callbacks (height/round against the current round, StateValidate,
 * StateCompare, MessageValidator, the lock-release stage) are left to the
 * caller: status != BH_BDLS_OK means Go rejects the message for certain;
 * BH_BDLS_OK means the signature layer and proof structure pass. The quorum
 * checks (2t+1 proofs to the proposed state, <select> proposal counts) use
 * the default Config.StateHash (BLAKE2b-256 of the state, consensus.go:41);
 * pass BH_BDLS_F_NO_QUORUM with a custom StateHash.
 *
 * sp_reason (optional unless BH_BDLS_F_GIVEN_REASONS): one byte per decoded
 * SignedProto, message by message in the order [outer, proofs..., LockRelease,
 * its proofs..., resync sub-messages...] (results[i].sp_first / sp_count):
 * BH_R_OK, a BH_R_* reject, or BH_SP_NOT_VERIFIED (signer not a participant,
 * or the outer version is wrong). These feed a verified-signature cache that
 * the unchanged ReceiveMessage then consults.
 * *sp_total (required) receives the number of decoded SignedProtos; with
 * sp_reason != NULL and sp_cap < *sp_total the call fails with BH_E_INVALID
 * before any device work (call again with a larger buffer). */
#define BH_BDLS_F_GIVEN_REASONS 1u /* sp_reason is INPUT (e.g. cache hits): no device work */
#define BH_BDLS_F_NO_QUORUM 2u     /* skip the StateHash-based quorum checks */
#define BH_SP_NOT_VERIFIED 255

#define BH_BDLS_OK 0
#define BH_BDLS_DECODE 1                    /* proto.Unmarshal(SignedProto) failed, :1212 */
#define BH_BDLS_VERSION 2                   /* ErrMessageVersion, :1218 */
#define BH_BDLS_UNKNOWN_PARTICIPANT 3       /* ErrMessageUnknownParticipant, :469 */
#define BH_BDLS_BAD_SIGNATURE 4             /* ErrMessageSignature, :486 */
#define BH_BDLS_MSG_DECODE 5                /* proto.Unmarshal(Message) failed, :490 */
#define BH_BDLS_UNKNOWN_TYPE 6              /* ErrMessageUnknownMessageType */
#define BH_BDLS_EMPTY_STATE 7               /* Err{Lock,Decide}EmptyState */
#define BH_BDLS_NOT_LEADER 8                /* Err{Lock,Select,Decide}NotSignedByLeader */
#define BH_BDLS_PROOF_UNKNOWN_PARTICIPANT 9 /* Err*ProofUnknownParticipant */
#define BH_BDLS_PROOF_BAD_SIGNATURE 10      /* ErrMessageSignature from a proof */
#define BH_BDLS_PROOF_DECODE 11             /* a proof's Message does not decode */
#define BH_BDLS_PROOF_TYPE_MISMATCH 12      /* Err*ProofTypeMismatch */
#define BH_BDLS_PROOF_HEIGHT_MISMATCH 13    /* Err*ProofHeightMismatch */
#define BH_BDLS_PROOF_ROUND_MISMATCH 14     /* Err*ProofRoundMismatch */
#define BH_BDLS_PROOF_INSUFFICIENT 15       /* Err{Lock,Select,Decide}ProofInsufficient */
#define BH_BDLS_SELECT_STATE_MISMATCH 16    /* ErrSelectStateMismatch */
#define BH_BDLS_SELECT_PROOF_EXCEEDED 17    /* ErrSelectProofExceeded */
#define BH_BDLS_LOCKRELEASE_EMPTY 18        /* ErrMessageIsEmpty (nil LockRelease) */

typedef struct bh_bdls_msg_result {
  int32_t status;            /* BH_BDLS_* */
  int32_t bad_sp;            /* SignedProto (relative to sp_first) that failed, or -1 */
  uint32_t type;             /* Message.Type (valid from status >= BH_BDLS_UNKNOWN_TYPE or OK) */
  uint32_t distinct_signers; /* distinct participants among the checked proofs */
  uint64_t height;           /* Message.Height */
  uint64_t round;            /* Message.Round */
  uint32_t sp_first;         /* first SignedProto of this message in sp_reason */
  uint32_t sp_count;
} bh_bdls_msg_result;

/* msgs/msg_off/msg_len: n raw SignedProto encodings (host). participants:
 * n_participants * 64 bytes, Identity = X || Y (Config.Participants order,
 * which defines roundLeader). curve: BH_CURVE_SECP256K1 or BH_CURVE_P256. */
int bh_bdls_preverify(int curve, const uint8_t *msgs, const uint64_t *msg_off,
                      const uint32_t *msg_len, size_t n, const uint8_t *participants,
                      size_t n_participants, uint32_t flags, bh_bdls_msg_result *results,
                      uint8_t *sp_reason, size_t sp_cap, size_t *sp_total);

/* ---- Fabric block pre-verification ------------------------------------------
 * Replaces the per-signature bccsp Verify calls of one block's validation
 * (core/committer/txvalidator/v20/validator.go:180-265, validateTx :297-453)
 * with ONE device batch: the serialized common.Block is decoded (protobuf-go
 * wire rules), and for every transaction
 *   - the creator signature over Envelope.payload by SignatureHeader.creator
 *     (core/common/validation/msgvalidation.go:26-64, checked at :274), and
 *   - for ENDORSER_TRANSACTIONs each endorsement over
 *     proposal_response_payload || endorser by the endorser
 *     (core/common/validation/statebased/validator_keylevel.go:246-260),
 *     de-duplicated per identity exactly as common/policies/policy.go:363-395
 *     SignatureSetToValidIdentities does (a later signature of an identity
 *     is checked only while no earlier one of it verified)
 * are verified with identity.Verify semantics (msp/identities.go:170-199:
 * SHA-256, or SHA3-256 with BH_FAB_F_SHA3; Fabric's low-S rule). Identities
 * (msp.SerializedIdentity: PEM X.509) resolve to P-256 keys through a
 * long-lived cache; one this library cannot resolve is reported, never
 * guessed. Checks that do not decide which signatures are verified
 * (CheckTxID, the proposal hash, channel / ledger state, policies) stay with
 * the unchanged validator, which consults the per-signature results.
 *
 * txs[i] (tx_cap >= number of transactions) and endorse[] (one byte per
 * endorsement, tx i's at [endorse_first, +endorse_count)); *n_tx and
 * *n_endorse are always set, and with too small buffers the call fails with
 * BH_E_INVALID before any device work. endorse[j]: BH_R_* when verified,
 * BH_FAB_E_DUPLICATE (skipped by the de-duplication), BH_FAB_E_BAD_IDENTITY,
 * or BH_SP_NOT_VERIFIED. */
#define BH_FAB_F_SHA3 1u      /* the MSPs' SignatureHashFamily is SHA3 */
#define BH_FAB_F_KEEP_KEYS 2u /* keys used >= 2 times get kept tables (BH_F_KEEP_KEYS) */
#define BH_FAB_F_DECODE_ONLY 4u /* decode, resolve and plan only: no device work, every
                                   signature BH_SP_NOT_VERIFIED (host-side structure checks) */

#define BH_FAB_OK 0                 /* every check below passed */
#define BH_FAB_ENVELOPE 1           /* Envelope does not unmarshal: INVALID_OTHER_REASON (validator.go:310) */
#define BH_FAB_PAYLOAD 2            /* Payload does not unmarshal: BAD_PAYLOAD (msgvalidation.go:257-261) */
#define BH_FAB_HEADER 3             /* validateCommonHeader failed: BAD_COMMON_HEADER (:264-269) */
#define BH_FAB_CREATOR_IDENTITY 4   /* creator not resolvable here (Go's DeserializeIdentity decides) */
#define BH_FAB_CREATOR_SIGNATURE 5  /* creator.Verify failed (or nil signature): BAD_CREATOR_SIGNATURE */
#define BH_FAB_TX 6                 /* endorser-transaction structure: INVALID_ENDORSER_TRANSACTION */
#define BH_FAB_UNSUPPORTED 7        /* CONFIG_UPDATE envelope: UNSUPPORTED_TX_PAYLOAD */
#define BH_FAB_E_DUPLICATE 253
#define BH_FAB_E_BAD_IDENTITY 254

typedef struct bh_fab_tx {
  int32_t status;           /* BH_FAB_*: the first failing check in the validator's order */
  int32_t type;             /* ChannelHeader.type (0 if the header did not decode) */
  uint32_t creator;         /* BH_R_* of the creator signature, or BH_SP_NOT_VERIFIED */
  uint32_t endorse_first;   /* this transaction's endorsements in endorse[] */
  uint32_t endorse_count;
  uint32_t valid_endorsers; /* |SignatureSetToValidIdentities(endorsement set)| */
} bh_fab_tx;

int bh_fabric_block_preverify(const uint8_t *block, size_t len, uint32_t flags, bh_fab_tx *txs,
                              size_t tx_cap, size_t *n_tx, uint8_t *endorse, size_t endorse_cap,
                              size_t *n_endorse);

/* bh_fabric_block_preverify plus, per signature, where its inputs lie in the
 * block: the keys of the caller's verified-signature cache (INTEGRATION.md
 * sections 4-5), consulted by the unchanged checkSignatureFromCreator
 * (msgvalidation.go:26-64) and SignatureSetToValidIdentities (policy.go:
 * 363-395) with exactly (identity, signed bytes, signature). refs[i] (i <
 * *n_tx) is transaction i's creator signature (identity = SignatureHeader.
 * creator, signed bytes = Envelope.payload, signature = Envelope.signature;
 * ident_len 0 when the transaction has no creator to check); refs[*n_tx + j]
 * is endorsement j (identity = endorser, signed bytes = proposal_response_
 * payload || endorser, the SignedData of validator_keylevel.go:246-260).
 * Offsets are byte offsets into `block`; reason repeats txs[i].creator /
 * endorse[j]. *n_ref = *n_tx + *n_endorse; ref_cap must cover it. */
typedef struct bh_fab_sigref {
  uint64_t ident_off, sig_off, msg_off, msg2_off;
  uint32_t ident_len, sig_len, msg_len, msg2_len; /* signed bytes: msg || msg2 */
  uint32_t reason;                                /* BH_R_*, BH_FAB_E_*, BH_SP_NOT_VERIFIED */
  uint32_t reserved;
} bh_fab_sigref;
int bh_fabric_block_preverify_refs(const uint8_t *block, size_t len, uint32_t flags,
                                   bh_fab_tx *txs, size_t tx_cap, size_t *n_tx, uint8_t *endorse,
                                   size_t endorse_cap, size_t *n_endorse, bh_fab_sigref *refs,
                                   size_t ref_cap, size_t *n_ref);

/* ---- signature sets: SignatureSetToValidIdentities as a batch ------------------
 * common/policies/policy.go:363-395, the batch point of every policy
 * evaluation (cauthdsl, implicit-meta sub-policies, the endorsement policy,
 * SigFilter, block signatures): for each signature set, in order, an entry
 * whose identity does not deserialize is skipped, an entry of an identity
 * already validated earlier in the set is skipped (de-duplication by Mspid +
 * Id, Id over the sanitized certificate), every other entry is verified with
 * identity.Verify (hash of data, then Verify, low-S). Sets are [set_first[k],
 * set_first[k+1]) (the last ends at n). result[i]: BH_R_* when verified,
 * BH_FAB_E_DUPLICATE, BH_FAB_E_BAD_IDENTITY, or BH_SP_NOT_VERIFIED;
 * valid_identities[k] = the number of identities the set yields. Flags:
 * BH_FAB_F_SHA3 / BH_FAB_F_KEEP_KEYS / BH_FAB_F_DECODE_ONLY. */
typedef struct bh_sd_batch { /* protoutil.SignedData {Identity, Data, Signature}, SoA */
  const uint8_t *identity;   /* msp.SerializedIdentity bytes */
  const uint64_t *identity_off;
  const uint32_t *identity_len;
  const uint8_t *data;       /* the signed bytes */
  const uint64_t *data_off;
  const uint32_t *data_len;
  const uint8_t *sig;        /* DER signatures */
  const uint64_t *sig_off;
  const uint32_t *sig_len;
} bh_sd_batch;
int bh_signature_sets_verify(const bh_sd_batch *b, size_t n, const uint32_t *set_first,
                             size_t n_sets, uint32_t flags, uint8_t *result,
                             uint32_t *valid_identities);

/* Orderer broadcast SigFilter (orderer/common/msgprocessor/sigfilter.go:50-80)
 * for n serialized common.Envelopes: EnvelopeAsSignedData
 * (protoutil/signeddata.go:60-86) then the one-signature set of the policy.
 * status[i]: BH_FAB_OK, BH_FAB_ENVELOPE, BH_FAB_PAYLOAD, BH_FAB_HEADER
 * ("Missing Header" / signature header), BH_FAB_CREATOR_IDENTITY,
 * BH_FAB_CREATOR_SIGNATURE; reason[i]: BH_R_* or BH_SP_NOT_VERIFIED. */
int bh_envelopes_preverify(const uint8_t *envs, const uint64_t *env_off, const uint32_t *env_len,
                           size_t n, uint32_t flags, int32_t *status, uint8_t *reason);

/* Block signatures (protoutil/blockutils.go:245-300 BlockSignatureVerifier,
 * non-BFT form, as orderer/common/cluster/util.go:300 VerifyBlockSignature and
 * the peer's gossip MCS run it) for n serialized blocks: per block the
 * SIGNATURES metadata's signature set, signed data = Metadata.value ||
 * signature_header || BlockHeaderBytes(header) (ASN.1 DER of number,
 * previous_hash, data_hash), de-duplicated as above. sig_reason[]:
 * one byte per MetadataSignature, block i's at [sig_first, +sig_count). */
#define BH_BLK_OK 0
#define BH_BLK_DECODE 1            /* block does not unmarshal or has no header */
#define BH_BLK_NO_SIGNATURES 2     /* "no signatures in block metadata" */
#define BH_BLK_METADATA 3          /* Metadata does not unmarshal */
#define BH_BLK_SIGNATURE_HEADER 4  /* a signature header does not unmarshal */
#define BH_BLK_IDENTIFIER_HEADER 5 /* BFT: an IdentifierHeader does not unmarshal */
#define BH_FAB_E_NOT_CONSENTER 252 /* BFT: identifier outside the consenter set (not in the set) */
typedef struct bh_blocksig_result {
  int32_t status;            /* BH_BLK_* */
  uint32_t sig_first;
  uint32_t sig_count;
  uint32_t valid_identities; /* identities the policy evaluation receives */
} bh_blocksig_result;
int bh_block_signatures_preverify(const uint8_t *blocks, const uint64_t *block_off,
                                  const uint32_t *block_len, size_t n, uint32_t flags,
                                  bh_blocksig_result *res, uint8_t *sig_reason, size_t sig_cap,
                                  size_t *sig_total);

/* BFT form (protoutil/blockutils.go:245-308 with bftEnabled, the V3_0 channel
 * capability, common/capabilities/channel.go:111; this fork registers BDLS as
 * consensus type "BFT", orderer/common/server/main.go:628). With
 * BH_BLK_F_BFT, a MetadataSignature whose signature_header is empty and whose
 * identifier_header is not is signed by the consenter with that identifier
 * (the FIRST cb.Consenter with Id == IdentifierHeader.identifier; identity =
 * marshalled msp.SerializedIdentity{MspId, Identity}) over Metadata.value ||
 * identifier_header || BlockHeaderBytes; an identifier outside the set is
 * skipped by Go (reported BH_FAB_E_NOT_CONSENTER, not part of the set's
 * de-duplication), and an IdentifierHeader that does not unmarshal fails the
 * block (BH_BLK_IDENTIFIER_HEADER). Without the flag (or with the signature
 * header present) this is bh_block_signatures_preverify. consenters may be
 * NULL (an empty set). */
#define BH_BLK_F_BFT 8u
typedef struct bh_consenter_set { /* cb.Consenter{Id, MspId, Identity}, SoA */
  const uint32_t *id;
  const uint8_t *msp_id;     /* MspId strings (not NUL-terminated) */
  const uint64_t *msp_id_off;
  const uint32_t *msp_id_len;
  const uint8_t *identity;   /* Identity bytes (PEM certificate) */
  const uint64_t *identity_off;
  const uint32_t *identity_len;
  size_t n;
} bh_consenter_set;
int bh_block_signatures_preverify_bft(const uint8_t *blocks, const uint64_t *block_off,
                                      const uint32_t *block_len, size_t n, uint32_t flags,
                                      const bh_consenter_set *consenters, bh_blocksig_result *res,
                                      uint8_t *sig_reason, size_t sig_cap, size_t *sig_total);

/* ---- X.509 certificate signatures ---------------------------------------------
 * Certificate i's signature against issuer key i (X || Y): Go crypto/x509
 * Certificate.CheckSignatureFrom for an ECDSA issuer (checkSignature: SHA-256
 * of the raw TBSCertificate, then ecdsa.VerifyASN1 -- cryptobyte-strict DER,
 * r, s in [1, n-1], NO low-S rule), the per-link check of the MSP's chain
 * validation (msp/mspimpl.go:717-722 cert.Verify, msp/cert.go:76-116). The
 * TBS bytes are hashed on the device straight out of the caller's buffer.
 * reason: BH_R_OK, BH_R_DER (signature not strict DER), BH_R_R_NONPOS /
 * BH_R_S_NONPOS (zero), BH_R_BAD_KEY, BH_R_R_RANGE / BH_R_S_RANGE, BH_R_MATH,
 * or BH_R_UNSUPPORTED (not ecdsa-with-SHA256, inner/outer algorithm mismatch,
 * or not a certificate this parser walks). */
int bh_verify_x509(const uint8_t *certs, const uint64_t *cert_off, const uint32_t *cert_len,
                   const uint8_t *issuer_pub, size_t n, uint8_t *bitmap, uint8_t *reason);

/* ---- device buffers on an initialised device (callers that keep batches
 * resident in HBM, e.g. bench.py; the library owns the HIP runtime so callers
 * never mix runtimes). Copies are synchronous on the device's stream. ---- */
int bh_dev_alloc(int device, size_t bytes, void **ptr);
int bh_dev_free(int device, void *ptr);
int bh_memcpy_h2d(int device, void *dst, const void *src, size_t bytes);
int bh_memcpy_d2h(int device, void *dst, const void *src, size_t bytes);
int bh_sync(int device); /* wait for all work queued on the device's library stream */

/* Deferred stage timing for pipelined callers: after bh_timing_begin, every
 * pass on `device` that is given no bh_timing records HIP events around its
 * stages on its launch stream WITHOUT synchronising; bh_timing_end waits for
 * those events and returns the stage times summed over the passes since
 * begin (routing counts and lanes of the last pass). */
int bh_timing_begin(int device);
int bh_timing_end(int device, bh_timing *timing);

/* ---- key registry ---------------------------------------------------------
 * Per device and curve, a persistent store of per-key fixed-base tables
 * (65 x 8 multiples of Q, 56 KiB per key in HBM). A record whose public key
 * is registered skips every doubling: u2 Q is 65 table additions. This is the
 * device-side counterpart of the reference's long-lived identities -- the
 * MSP identity cache (msp/cache/cache.go) for Fabric, the fixed participant
 * set (consensus.go:456-466, Config.Participants) for BDLS. Verification
 * results never depend on the registry (same bitmap and reasons with or
 * without it); only the route and the time do.
 * capacity: tables per (device, curve); bh_keys_register / BH_F_KEEP_KEYS
 * reserve 65536 on first use when not reserved before. Entries persist until
 * bh_keys_clear; once full, new keys take the per-batch path. */
int bh_keys_reserve(int device, int curve, size_t capacity);
/* Import and register n keys (host pointer, n * 64 bytes X || Y). status
 * (optional, n bytes): 0 registered (or already present), BH_R_BAD_KEY not a
 * valid curve point, 255 registry full. Synchronous. */
int bh_keys_register(int device, int curve, const uint8_t *pub, size_t n, uint8_t *status);
int bh_keys_clear(int device, int curve);
int bh_keys_count(int device, int curve, size_t *count);

#ifdef __cplusplus
}
#endif
#endif /* BDLS_HIP_H */
