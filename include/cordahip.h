/* cordahip.h — C-ABI of libcordahip.so, the MI355X batch signature and
 * transaction-id verification engine for Corda's hot path.
 *
 * Drop-in boundary. Every entry point is plain C: pointers,
 * sizes, status codes; no C++ types or exceptions cross it, so a JNI shim (see
 * INTEGRATION.md) or ctypes binds it directly. The entry points replace:
 *
 *   cordahip_sig_submit / cordahip_sig_verify
 *       -> Crypto.isValid(scheme, key, sig, clear)   core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541
 *          Crypto.doVerify(scheme, key, sig, clear)  Crypto.kt:472-483
 *          (one call per signature today, through the JCA SPI at Crypto.kt:537-540;
 *           here: one call per BATCH, per-lane status instead of throw/false)
 *   cordahip_ed25519_verify_device / _host
 *       -> the EDDSA_ED25519_SHA512 lane of the above (Crypto.kt:119-132), dense layout
 *   cordahip_ed25519_sign_device
 *       -> Crypto.doSign(EDDSA_ED25519_SHA512, ...) (Crypto.kt:380-400) and
 *          deriveKeyPairFromEntropy (Crypto.kt:733-739): corpus generation only
 *   cordahip_tx_ids (tx id = Merkle root of component hashes)
 *       -> WireTransaction.id (WireTransaction.kt:48) = MerkleTree.getMerkleTree(
 *          availableComponentHashes).hash (MerkleTree.kt:27-66, MerkleTransaction.kt:69)
 *   cordahip_signed_tx_verify / cordahip_tx_submit
 *       -> SignedTransaction.checkSignaturesAreValid (SignedTransaction.kt:95-100)
 *          + the tx.id recomputation of verifySignatures (:70-85); signer coverage
 *          (getMissingSignatures :102-108) stays with the caller, see INTEGRATION.md.
 *          The _submit forms return a ticket at once: the caller (a Quasar fiber in
 *          ResolveTransactionsFlow.call, ResolveTransactionsFlow.kt:97-122, on the
 *          single Node thread) suspends on it instead of blocking the thread.
 *
 * Result contract: a return value < 0 means the whole call failed (the caller
 * falls back to the JVM path for that batch); per-lane outcomes are DATA in
 * status[] (CORDAHIP_STATUS_*), never return codes.
 *
 * Ownership: the caller owns every host buffer and must leave it untouched
 * until cordahip_wait()/poll() reports the ticket done. Buffers from
 * cordahip_alloc_pinned() are page-locked (hipHostMalloc) and are the fast
 * path for host batches. The library owns device memory and HIP streams.
 * A context is thread-safe: submit/wait/poll from any thread.
 */
#ifndef CORDAHIP_H
#define CORDAHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CORDAHIP_ABI_VERSION 4u

/* ---- per-lane statuses (status[i]) ------------------------------------- */
#define CORDAHIP_STATUS_OK 0            /* isValid -> true;  doVerify -> true                         */
#define CORDAHIP_STATUS_BAD_SIG 1       /* isValid -> false; doVerify -> SignatureException            */
#define CORDAHIP_STATUS_MALFORMED_SIG 2 /* SignatureException from the engine (bad length / DER)       */
#define CORDAHIP_STATUS_BAD_KEY 3       /* key decode failed (IllegalArgumentException at key build)   */
#define CORDAHIP_STATUS_UNSUPPORTED 4   /* IllegalArgumentException: unsupported scheme (Crypto.kt:474)*/
#define CORDAHIP_STATUS_EMPTY 5         /* IllegalArgumentException: empty sig / clear (Crypto.kt:475) */

/* ---- return codes -------------------------------------------------------- */
#define CORDAHIP_SUCCESS 0
#define CORDAHIP_ERR_INVALID_ARG (-1)
#define CORDAHIP_ERR_HIP (-2)
#define CORDAHIP_ERR_NO_DEVICE (-3)
#define CORDAHIP_ERR_OUT_OF_MEMORY (-4)
#define CORDAHIP_ERR_TIMEOUT (-5)
#define CORDAHIP_ERR_UNKNOWN_TICKET (-6)
#define CORDAHIP_ERR_NOT_IMPLEMENTED (-7)
/* -8 CORDAHIP_ERR_BUFFER_TOO_SMALL: see cordahip_kryo_encode */

/* ---- signature schemes = Corda SignatureScheme.schemeNumberID ------------ */
#define CORDAHIP_SCHEME_RSA_SHA256 1             /* Crypto.kt:77  (not on GPU -> UNSUPPORTED lane) */
#define CORDAHIP_SCHEME_ECDSA_SECP256K1_SHA256 2 /* Crypto.kt:92  */
#define CORDAHIP_SCHEME_ECDSA_SECP256R1_SHA256 3 /* Crypto.kt:106 */
#define CORDAHIP_SCHEME_EDDSA_ED25519_SHA512 4   /* Crypto.kt:120 */
#define CORDAHIP_SCHEME_SPHINCS256_SHA256 5      /* Crypto.kt:140 (not on GPU -> UNSUPPORTED lane) */

typedef struct cordahip_ctx cordahip_ctx;

uint32_t cordahip_abi_version(void);
const char* cordahip_strerror(int code);

/* device_mask: bit d selects visible HIP device d; 0 = all visible devices. */
int cordahip_init(uint32_t device_mask, cordahip_ctx** out);
void cordahip_shutdown(cordahip_ctx* ctx);
int cordahip_device_count(const cordahip_ctx* ctx);

/* Device memory (ABI 4). cordahip_device_mem: the bytes the library holds on
 * `device`'s GPU now and at most so far (workspaces, stages, fixed tables), and
 * its budget. The budget (CORDAHIP_DEVICE_MEM_BUDGET at cordahip_init, bytes
 * with an optional K/M/G suffix; default 128 GiB, at most 90% of the device)
 * sizes the verification workspaces -- Ed25519 45% (+20% for the pipelines'
 * second slot), ECDSA 15%; a smaller budget only costs extra launches. The
 * batch-proportional buffers (stages, id buffers) follow the batches. Buffers
 * are grow-only while a device is busy; after CORDAHIP_IDLE_RELEASE_MS (default
 * 30000; 0: never) without a call they are released, as cordahip_trim does now
 * (it waits for the calls in progress). INTEGRATION.md §6. */
int cordahip_device_mem(cordahip_ctx* ctx, int device, uint64_t* in_use, uint64_t* peak, uint64_t* budget);
int cordahip_trim(cordahip_ctx* ctx);

int cordahip_alloc_pinned(cordahip_ctx* ctx, size_t bytes, void** host);
int cordahip_free_pinned(cordahip_ctx* ctx, void* host);

/* ---- generic signature batch (host memory) ------------------------------ *
 * Variable-length fields are CSR: item i's key is key[key_off[i] .. key_off[i+1]).
 * Every CSR array in this header is CHECKED (ABI 4): offsets non-decreasing, the
 * last one within the buffer length the batch declares (key_bytes, sig_bytes,
 * msg_bytes, leaf_bytes_len, n_items, ntok), and each level's range inside the
 * next level's declared count (a transaction's leaves < nleaves, items < n_items,
 * signatures < nsig): the library reads no array past the entries its declared
 * count implies ([n+1] offsets for n entries). A violation fails the batch
 * with CORDAHIP_ERR_INVALID_ARG, never a read outside the caller's buffers:
 * transaction-level batches are checked whole before anything is enqueued; a
 * generic signature batch is checked lane by lane as its chunks are classified
 * (earlier chunks may then have written their statuses; the result is the error).
 * The context stays usable after INVALID_ARG.
 * Key encodings: Ed25519 = the 32-byte A (Kryo wire form, Kryo.kt:386); ECDSA =
 * SEC1 point (the SPKI BIT STRING payload, Crypto.kt:348-355).
 * verdict (optional): bit (i % 64) of word (i / 64) = (status[i] == OK).
 * flags: 0 = Crypto.doVerify semantics (Crypto.kt:472-483: empty signature or
 * clear data -> EMPTY); CORDAHIP_FLAG_IS_VALID = Crypto.isValid semantics
 * (Crypto.kt:534-541: no emptiness checks; an empty clear data is hashed like
 * any other message and may verify, an empty signature is MALFORMED_SIG at the
 * engine). Lanes are sharded over every context device (contiguous, 64-aligned
 * shards of each scheme's lanes; cordahip_shard_range).                      */
#define CORDAHIP_FLAG_IS_VALID 1u
typedef struct {
  uint64_t n;
  const uint8_t* scheme; /* [n] CORDAHIP_SCHEME_* */
  const uint8_t* key;
  const uint64_t* key_off; /* [n+1] */
  const uint8_t* sig;
  const uint64_t* sig_off; /* [n+1] */
  const uint8_t* msg;
  const uint64_t* msg_off; /* [n+1] */
  uint8_t* status;         /* [n] out */
  uint64_t* verdict;       /* [(n+63)/64] out, may be NULL */
  uint32_t flags;          /* CORDAHIP_FLAG_* */
  uint64_t key_bytes;      /* ABI 4: bytes at key; key_off[n] <= key_bytes */
  uint64_t sig_bytes;      /* bytes at sig */
  uint64_t msg_bytes;      /* bytes at msg */
} cordahip_sig_batch;

/* Tickets: every *_submit queues the batch on the context's worker pool and
 * returns at once. cordahip_wait() returns the batch's result code and RELEASES
 * the ticket (a second wait gives CORDAHIP_ERR_UNKNOWN_TICKET); cordahip_poll()
 * only reports progress, so every ticket must be waited on once (shutdown
 * waits for and releases the rest). The descriptor is copied at submit; the
 * buffers it points to stay the caller's and must stay untouched until wait. */
int cordahip_sig_submit(cordahip_ctx* ctx, const cordahip_sig_batch* batch, uint64_t* ticket);
/* timeout_ns < 0: wait forever; CORDAHIP_ERR_TIMEOUT keeps the ticket. */
int cordahip_wait(cordahip_ctx* ctx, uint64_t ticket, int64_t timeout_ns);
/* 1 = done (result retrievable with wait), 0 = pending, < 0 = error */
int cordahip_poll(cordahip_ctx* ctx, uint64_t ticket);
/* synchronous submit + wait */
int cordahip_sig_verify(cordahip_ctx* ctx, const cordahip_sig_batch* batch);

/* ---- dense Ed25519 paths -------------------------------------------------- *
 * keys n*32 B, sigs n*64 B (R || S), msgs n*msg_len B, all row-major.
 * _device: pointers are device (HBM) memory on `device`; 16-byte aligned;
 *          enqueued on hip_stream (a hipStream_t; NULL = the device's null
 *          stream, with HIP's usual null-stream ordering); asynchronous w.r.t.
 *          the host, ordered after earlier work on that stream.
 * _host:   host pointers (pinned recommended); shards over all context devices,
 *          pipelines H2D copy / kernel / D2H copy in chunks; synchronous.   */
int cordahip_ed25519_verify_device(cordahip_ctx* ctx, int device, const void* d_keys, const void* d_sigs,
                                   const void* d_msgs, uint32_t msg_len, uint64_t n, void* d_status,
                                   void* d_verdict, void* hip_stream);
int cordahip_ed25519_verify_host(cordahip_ctx* ctx, const uint8_t* keys, const uint8_t* sigs, const uint8_t* msgs,
                                 uint32_t msg_len, uint64_t n, uint8_t* status, uint64_t* verdict);

/* ---- dense ECDSA path (secp256k1 = 2 and P-256 = 3 mixed) ------------------ *
 * scheme[n]; keys in 65-byte slots (SEC1 04||X||Y or 02/03||X) + key_len[n];
 * DER signatures in 72-byte slots + sig_len[n] (72 = the longest DER encoding of
 * r, s < 2^256); msgs n*msg_len. Device memory; lanes are partitioned by curve on
 * the device (one curve per wavefront), status and verdict come back in input order.
 * A lane with sig_len > 72 does not fit its slot: it is MALFORMED_SIG here (EMPTY
 * first under doVerify rules), without reading past the slot. BouncyCastle would
 * say BAD_SIG for such a signature when its DER is well formed (an INTEGER of more
 * than 33 bytes is >= n): use the generic batch (cordahip_sig_verify), which
 * decides those lanes by the DER rules, for BC parity on over-long signatures. */
int cordahip_ecdsa_verify_device(cordahip_ctx* ctx, int device, const void* d_scheme, const void* d_keys,
                                 const void* d_key_len, const void* d_sigs, const void* d_sig_len, const void* d_msgs,
                                 uint32_t msg_len, uint64_t n, void* d_status, void* d_verdict, void* hip_stream);

/* ---- streaming mixed-scheme drain (verifier-module queue) ----- *
 * Replaces the per-request Crypto.isValid calls a verifier would make for a
 * queue of mixed-scheme requests (Crypto.kt:534-541; the out-of-process
 * verifier's request loop, verifier/.../Verifier.kt:58-75).
 * The producer writes requests straight into the two dense host layouts
 * (pinned memory from cordahip_alloc_pinned, or the copies are not
 * asynchronous): an Ed25519 section (as cordahip_ed25519_verify_host) and an
 * ECDSA section (as cordahip_ecdsa_verify_device, 65/72-byte slots). Each
 * context device takes a contiguous shard of both sections and streams it in
 * chunks of up to 2^23 lanes through 3 device buffer sets on three HIP
 * streams (every H2D on one copy stream; each section's kernels and status
 * D2H on its own stream, so a chunk's ECDSA kernels run beside its Ed25519
 * kernels), so the H2D copy of chunk k+1, the kernels of chunk k and the
 * status D2H of chunk k-1 overlap. All of the batch's host buffers, statuses
 * included, must be pinned. Synchronous; statuses land in ed_status /
 * ec_status.                                                                  */
typedef struct {
  uint64_t n_ed;
  const uint8_t* ed_keys; /* [n_ed*32] */
  const uint8_t* ed_sigs; /* [n_ed*64] */
  const uint8_t* ed_msgs; /* [n_ed*ed_msg_len] */
  uint32_t ed_msg_len;
  uint8_t* ed_status;     /* [n_ed] out */
  uint64_t n_ec;
  const uint8_t* ec_scheme;  /* [n_ec] 2 or 3 */
  const uint8_t* ec_keys;    /* [n_ec*65] SEC1 in 65-byte slots */
  const uint8_t* ec_key_len; /* [n_ec] */
  const uint8_t* ec_sigs;    /* [n_ec*72] DER in 72-byte slots */
  const uint8_t* ec_sig_len; /* [n_ec] */
  const uint8_t* ec_msgs;    /* [n_ec*ec_msg_len] */
  uint32_t ec_msg_len;
  uint8_t* ec_status;        /* [n_ec] out */
} cordahip_stream_batch;
int cordahip_stream_verify(cordahip_ctx* ctx, const cordahip_stream_batch* batch);

/* RFC 8032 keygen + sign from 32-byte seeds (device memory): corpus generation. */
int cordahip_ed25519_sign_device(cordahip_ctx* ctx, int device, const void* d_seeds, const void* d_msgs,
                                 uint32_t msg_len, uint64_t n, void* d_pubs, void* d_sigs, void* hip_stream);

/* ECDSA keygen + sign (device memory), corpus generation: per lane scheme 2/3,
 * d = SHA-256(seed) mod n, k = SHA-256(seed || msg[:64]) mod n; writes the
 * uncompressed SEC1 key (65-byte slot, key_len = 65) and the DER signature
 * (72-byte slot + sig_len). Not a production signer (deterministic synthetic nonce). */
int cordahip_ecdsa_sign_device(cordahip_ctx* ctx, int device, const void* d_scheme, const void* d_seeds,
                               const void* d_msgs, uint32_t msg_len, uint64_t n, void* d_keys, void* d_key_len,
                               void* d_sigs, void* d_sig_len, void* hip_stream);

/* ---- transaction ids and SignedTransaction batches ----------------------- */
/* tx-level statuses (tx_status[t]) in addition to the lane statuses above */
#define CORDAHIP_TX_NO_LEAVES 6     /* MerkleTreeException: empty component list (MerkleTree.kt:49-50) */
#define CORDAHIP_TX_NO_SIGNATURES 7 /* IllegalArgumentException: require(sigs.isNotEmpty()) (SignedTransaction.kt:37-39) */

/* Leaves are the serialised components of each WireTransaction, in
 * availableComponents order (MerkleTransaction.kt:51-62), each including the
 * "corda\0\0\1" Kryo header (Kryo.kt:101); the host serialises, the GPU hashes. */
typedef struct {
  uint64_t ntx;
  const uint8_t* leaf_bytes;
  const uint64_t* leaf_off;    /* [nleaves+1] into leaf_bytes */
  const uint64_t* tx_leaf_off; /* [ntx+1] leaves of tx t: [tx_leaf_off[t], tx_leaf_off[t+1]) */
  uint8_t* txid;               /* [ntx*32] out: WireTransaction.id (SecureHash bytes) */
  uint8_t* tx_status;          /* [ntx] out: OK, NO_LEAVES (ids) / first failing lane status (signed tx) */
  uint64_t nleaves;            /* ABI 4: leaves (leaf_off has nleaves+1 entries); tx_leaf_off[ntx] <= nleaves */
  uint64_t leaf_bytes_len;     /* bytes at leaf_bytes */
} cordahip_txid_batch;
int cordahip_tx_ids(cordahip_ctx* ctx, const cordahip_txid_batch* batch);

/* SignedTransaction.checkSignaturesAreValid over many transactions: every
 * signature is verified over its transaction's recomputed id; first_bad_sig[t]
 * is the index (within tx t, list order) of the signature whose exception the
 * reference would throw first, -1 if none. Signer coverage
 * (getMissingSignatures, CompositeKey.isFulfilledBy) stays with the caller. */
typedef struct {
  cordahip_txid_batch tx;
  const uint64_t* tx_sig_off; /* [ntx+1] signatures of tx t */
  const uint8_t* scheme;      /* [nsig] per signature, CSR key/sig as in cordahip_sig_batch */
  const uint8_t* key;
  const uint64_t* key_off;
  const uint8_t* sig;
  const uint64_t* sig_off;
  uint8_t* sig_status;    /* [nsig] out */
  int64_t* first_bad_sig; /* [ntx] out */
  uint64_t nsig;          /* ABI 4: signatures (key_off / sig_off have nsig+1 entries); tx_sig_off[ntx] <= nsig */
  uint64_t key_bytes;     /* bytes at key */
  uint64_t sig_bytes;     /* bytes at sig */
} cordahip_signed_tx_batch;
int cordahip_signed_tx_verify(cordahip_ctx* ctx, const cordahip_signed_tx_batch* batch);

/* Ticketed forms of cordahip_signed_tx_verify / cordahip_tx_ids (SURVEY §8b
 * cordahip_tx_submit): same results, completed through cordahip_wait/poll. */
int cordahip_tx_submit(cordahip_ctx* ctx, const cordahip_signed_tx_batch* batch, uint64_t* ticket);
int cordahip_txid_submit(cordahip_ctx* ctx, const cordahip_txid_batch* batch, uint64_t* ticket);

/* Device-resident dense variant (all Ed25519, 32-byte keys, 64-byte sigs;
 * every array in HBM on `device`): K3 leaf hashes -> K4 Merkle roots ->
 * txid gather -> K1 verify -> K5 per-tx reduce, all on hip_stream. */
int cordahip_signed_tx_verify_ed25519_device(cordahip_ctx* ctx, int device, const void* d_leaf_bytes,
                                             const void* d_leaf_off, uint64_t nleaves, const void* d_tx_leaf_off,
                                             uint64_t ntx, const void* d_tx_sig_off, const void* d_keys,
                                             const void* d_sigs, uint64_t nsig, void* d_txid, void* d_tx_status,
                                             void* d_first_bad, void* d_sig_status, void* hip_stream);

/* FilteredTransaction.verify over many filtered transactions:
 *   FilteredTransaction.verify   core/.../transactions/MerkleTransaction.kt:134-140
 *   PartialMerkleTree.verify     core/.../crypto/PartialMerkleTree.kt:132-158
 * Per filtered tx t: the FilteredLeaves' serialised components (leaf CSR exactly
 * as in cordahip_txid_batch; the GPU hashes them = availableComponentHashes),
 * the PartialMerkleTree as its post-order token stream tok[k] (0 IncludedLeaf,
 * 1 Leaf, 2 Node) with tok_hash[k*32 .. k*32+32) the hash of token k (ignored
 * for Node), and the claimed rootHash. tx_status[t]: OK (verify() == true),
 * BAD_SIG (verify() == false), CORDAHIP_TX_NO_LEAVES (MerkleTreeException,
 * no included leaves), CORDAHIP_TX_BAD_TREE (the token stream is not a tree:
 * no PartialMerkleTree serialises to it). */
#define CORDAHIP_TX_BAD_TREE 8
typedef struct {
  uint64_t ntx;
  const uint8_t* leaf_bytes;
  const uint64_t* leaf_off;    /* [nleaves+1] */
  const uint64_t* tx_leaf_off; /* [ntx+1] */
  const uint8_t* tok;          /* [ntok] */
  const uint8_t* tok_hash;     /* [ntok*32] */
  const uint64_t* tx_tok_off;  /* [ntx+1] */
  const uint8_t* root;         /* [ntx*32] claimed Merkle roots (FilteredTransaction.rootHash) */
  uint8_t* tx_status;          /* [ntx] out */
  uint64_t nleaves;            /* ABI 4: leaves (leaf_off has nleaves+1 entries) */
  uint64_t leaf_bytes_len;     /* bytes at leaf_bytes */
  uint64_t ntok;               /* tokens at tok (and 32-byte hashes at tok_hash) */
} cordahip_filtered_tx_batch;
int cordahip_filtered_tx_verify(cordahip_ctx* ctx, const cordahip_filtered_tx_batch* batch);
int cordahip_filtered_tx_submit(cordahip_ctx* ctx, const cordahip_filtered_tx_batch* batch, uint64_t* ticket);

/* ---- native Kryo leaf encoder ------------------------- *
 * The Merkle leaf of a transaction component is SHA-256 of its p2p Kryo bytes:
 *   serializedHash(x) = p2PKryo().withoutReferences { x.serialize(kryo).hash }
 *       core/.../transactions/MerkleTransaction.kt:16-18
 *   serialize = "corda\0\0\1" header + kryo.writeClassAndObject(x)
 *       core/.../serialization/Kryo.kt:101,165-176
 * cordahip_kryo_encode writes those preimages natively (no JVM re-serialisation)
 * for the component kinds whose wire form is fixed by Kryo 4.0.0's published
 * format plus Corda's own serializers; any other component travels as a RAW,
 * already-serialised leaf. Output is the leaf CSR cordahip_tx_ids consumes.
 * Kinds and their bytes after the header (varint = Kryo writeVarInt(x, true)):
 *   RAW            data[len] copied verbatim (a complete leaf, header included)
 *   CHAR/SHORT/INT/LONG/BYTE/BOOLEAN/FLOAT/DOUBLE  (boxed primitive, Kryo's
 *                  default registrations 5/6/0/7/4/3/2/8): varint(id + 2), then
 *                  the value big-endian in 2/2/4/8/1/1/4/8 bytes (value: bits)
 *   STRING         varint(1 + 2), Output.writeString of the UTF-16 code units
 *                  data[0..2*len) (little-endian u16): ASCII form for 2..63 ASCII
 *                  chars, else UTF-8 length + modified UTF-8
 *   ED25519_KEY    varint(class_id + 2), varint(32), A (Ed25519PublicKeySerializer,
 *                  Kryo.kt:383-393); data = the 32-byte A
 *   PUBLIC_KEY     varint(class_id + 2), varint(len), key.encoded (PublicKeySerializer,
 *                  Kryo.kt:441-451, BCEC/BCRSA/SPHINCS keys); data = X.509 SPKI DER
 *   KOTLIN_OBJECT  varint(NAME + 2 = 1), varint(name id 0), writeString(class
 *                  name) and no body (CordaClassResolver.registerImplicit's
 *                  KotlinObjectSerializer, CordaClassResolver.kt:76-99), e.g.
 *                  "net.corda.core.contracts.TransactionType$General"; data =
 *                  the class name as UTF-16 code units (len = chars)
 *   PARTY          the notary Party (identity/Party.kt): NAME registration of
 *                  "net.corda.core.identity.Party", CompatibleFieldSerializer
 *                  (EXTENDED names, DefaultKryoCustomizer.kt:56-58) over
 *                  AbstractParty.owningKey (key class + writeBytesWithLength) and
 *                  Party.name (X500NameSerializer, Kryo.kt:615-624); data = the
 *                  X.500 name's DER (self-delimiting) followed by the key bytes
 *                  (A, or the SPKI DER); class_id = X500Name's registration id;
 *                  value = the key class's registration id
 *   ISSUE_COMMAND  Command(value = an issue command data class with one Long
 *                  `nonce`, signers = Arrays.asList(keys)) as
 *                  TransactionBuilder.addCommand(data, vararg keys) builds it
 *                  (TransactionBuilder.kt:124, Structures.kt:285, Cash.kt:148);
 *                  data = u8 class-name length, the command data's binary class
 *                  name, u8 key count, per key u16 LE registration id, u16 LE
 *                  length, key bytes; class_id = java.util.Arrays$ArrayList's
 *                  registration id (ArraysAsListSerializer); value = the nonce
 *   CASH_STATE     TransactionState<Cash.State> -- the output of a cash issue
 *                  (Cash.generateIssue, Cash.kt:166-167; Structures.kt:95-117,
 *                  132,268; Cash.kt:35,62,92-103; Amount.kt:37): TransactionState
 *                  (data, encumbrance, notary) > Cash.State (amount, contract =
 *                  CASH_PROGRAM_ID, exitKeys = {owner key, issuer key},
 *                  owner, participants = [owner]) > Amount(quantity,
 *                  displayTokenSize = 10^-digits, Issued(PartyAndReference(
 *                  issuer, reference), Currency)). data = issuer party, u8
 *                  reference length, reference bytes, owner party, notary party,
 *                  u8 currency-code length, the code (ASCII), i8 the currency's
 *                  fraction digits, the 32-byte legalContractReference
 *                  (SHA-256 of Cash's legal-prose URL), u8 flags (bit 0:
 *                  encumbrance present), i32 LE encumbrance; a party = u16 LE key
 *                  registration id, u16 LE key length, key bytes, u16 LE X.500
 *                  name length, the name's DER (length 0 = AnonymousParty, e.g.
 *                  CashIssueFlow's anonymised recipient; the notary must be a
 *                  Party); class_id = X500Name's registration id; value = the
 *                  quantity (pennies)
 * Field values go through OutputChunked (1024-byte chunks + a zero chunk) as
 * Kryo 4.0.0's CompatibleFieldSerializer writes them, nested serializers'
 * flushes cutting the enclosing fields' chunks (kryo.cpp). PARTY / ISSUE_COMMAND
 * / CASH_STATE are restated from Kryo 4.0.0 / kryo-serializers 0.41 published
 * sources: PARITY
 * UNPINNED (no JVM here), except the Ed25519 key bytes inside them, which the
 * reference's own serialised keys pin (tests/golden/kryo_key_vectors.json).
 * class_id = kryo.getRegistration(cls).id on the node (registration order of
 * DefaultKryoCustomizer.kt is fixed per build; the JVM reads it once).
 * off[0..n] receives the CSR offsets; returns CORDAHIP_ERR_BUFFER_TOO_SMALL with
 * off[n] = the bytes needed when cap is too small, and CORDAHIP_ERR_INVALID_ARG
 * at the first invalid item -- `out` (and off) are then left partly written:
 * the leaves before that item are in place. Host-only: no device work. */
#define CORDAHIP_ERR_BUFFER_TOO_SMALL (-8)
#define CORDAHIP_KRYO_RAW 0
#define CORDAHIP_KRYO_CHAR 1
#define CORDAHIP_KRYO_SHORT 2
#define CORDAHIP_KRYO_INT 3
#define CORDAHIP_KRYO_LONG 4
#define CORDAHIP_KRYO_BYTE 5
#define CORDAHIP_KRYO_BOOLEAN 6
#define CORDAHIP_KRYO_FLOAT 7
#define CORDAHIP_KRYO_DOUBLE 8
#define CORDAHIP_KRYO_STRING 9
#define CORDAHIP_KRYO_ED25519_KEY 10
#define CORDAHIP_KRYO_PUBLIC_KEY 11
#define CORDAHIP_KRYO_KOTLIN_OBJECT 12
#define CORDAHIP_KRYO_PARTY 13
#define CORDAHIP_KRYO_ISSUE_COMMAND 14
#define CORDAHIP_KRYO_CASH_STATE 15
typedef struct {
  uint32_t kind;       /* CORDAHIP_KRYO_* */
  uint32_t class_id;   /* Kryo registration id (ED25519_KEY, PUBLIC_KEY) */
  int64_t value;       /* primitive kinds: the value (FLOAT / DOUBLE: the IEEE bits) */
  const uint8_t* data; /* RAW / STRING / key / class-name payload */
  uint64_t len;        /* bytes (RAW, keys) or UTF-16 code units (STRING, KOTLIN_OBJECT) */
} cordahip_kryo_item;
int cordahip_kryo_encode(const cordahip_kryo_item* items, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* off);

/* The same leaf preimages computed on the GPU, for components whose payloads
 * are already in device memory (a transaction batch's ids then need neither
 * host serialisation nor leaf bytes over PCIe). d_items: n items in device
 * memory whose `data` are device pointers; group: the items come as records of
 * `group` components (e.g. the 5 of a cash-issue transaction) -- a thread
 * mapping hint, 1 = none. Writes d_off[0..n] (uint64, the CSR offsets; d_off[n]
 * = the bytes of all leaves) and d_status[i] (uint8): 0 written, 1 invalid item
 * (as cordahip_kryo_encode would reject it; size 0), 2 not written because it
 * ends beyond cap. Enqueued on hip_stream, asynchronous; the caller reads
 * d_off[n] / d_status when it needs them. Same encoder as cordahip_kryo_encode
 * (corda_amd/csrc/kryo_core.hpp): bit-identical leaves; items of one shape
 * (equal structure, kryo_template.hpp) are written from a template traced once
 * per shape. d_out NULL: sizes and offsets only (statuses 0 / 1). n < 2^31 - 1
 * per call. Device scratch (grow-only, per device): 16 B per item, ~18 MB of
 * shape table and templates, 56 MB of level buffers for the items written
 * without a template. */
int cordahip_kryo_encode_device(cordahip_ctx* ctx, int device, const void* d_items, uint64_t n, uint32_t group,
                                void* d_out, uint64_t cap, void* d_off, void* d_status, void* hip_stream);

/* ---- component-level SignedTransaction batches (SURVEY §8b + §8f rank 4) ---- *
 * cordahip_signed_tx_verify with each transaction's COMPONENTS instead of their
 * serialised leaves: the JVM hands over the Kryo items of availableComponents
 * (MerkleTransaction.kt:51-62) and the GPU writes the leaf preimages
 * (serializedHash, MerkleTransaction.kt:16-18; the encoder of
 * cordahip_kryo_encode_device) ahead of K3 / K4, so tx ids need no JVM
 * re-serialisation and PCIe carries the components (~540 B per cash-issue
 * transaction: 160 B of items, 379 B of payload) instead of the leaves
 * (1,717 B). Once a device's component batches need no new template and no
 * direct encoder, it runs a templates-only encoder chain; a call that then
 * meets a new shape runs again with the full chain before it returns (same
 * outputs, about twice the time for that call). Replaces the same reference
 * calls as cordahip_tx_submit: SignedTransaction.checkSignaturesAreValid
 * (SignedTransaction.kt:95-100) + the id of verifySignatures (:70-85,
 * WireTransaction.kt:48).
 * items[i].data is an OFFSET into `payload` (not a pointer); any number of
 * items may share a payload (the notary Party, TransactionType). The payload
 * crosses PCIe as a growing prefix, slice by slice: laid out in transaction
 * order (shared payloads first) the first slice's copy stays short. An item
 * whose payload runs past payload_len, or that cordahip_kryo_encode would
 * reject, makes its transaction CORDAHIP_TX_BAD_COMPONENT (its id is not
 * computed; serialise that transaction on the JVM and use RAW leaves).
 * Signature fields, outputs and statuses as in cordahip_signed_tx_batch.     */
#define CORDAHIP_TX_BAD_COMPONENT 9
typedef struct {
  uint64_t ntx;
  const cordahip_kryo_item* items; /* [nitems] components, tx by tx, availableComponents order */
  const uint64_t* tx_item_off;     /* [ntx+1] items of tx t: [tx_item_off[t], tx_item_off[t+1]) */
  const uint8_t* payload;          /* item payloads (data = offsets into it) */
  uint64_t payload_len;
  uint8_t* txid;      /* [ntx*32] out */
  uint8_t* tx_status; /* [ntx] out */
  uint64_t n_items;   /* ABI 4: records at items; tx_item_off[ntx] <= n_items */
} cordahip_txcomp_batch;
typedef struct {
  cordahip_txcomp_batch tx;
  const uint64_t* tx_sig_off; /* [ntx+1] */
  const uint8_t* scheme;      /* [nsig] */
  const uint8_t* key;
  const uint64_t* key_off;
  const uint8_t* sig;
  const uint64_t* sig_off;
  uint8_t* sig_status;    /* [nsig] out */
  int64_t* first_bad_sig; /* [ntx] out */
  uint64_t nsig;          /* ABI 4: signatures (key_off / sig_off have nsig+1 entries) */
  uint64_t key_bytes;     /* bytes at key */
  uint64_t sig_bytes;     /* bytes at sig */
} cordahip_signed_txcomp_batch;
int cordahip_signed_txcomp_verify(cordahip_ctx* ctx, const cordahip_signed_txcomp_batch* batch);
int cordahip_txcomp_submit(cordahip_ctx* ctx, const cordahip_signed_txcomp_batch* batch, uint64_t* ticket);

/* Device-resident component-level variant (all Ed25519, 32-byte keys, 64-byte
 * sigs; every array in HBM on `device`, items[i].data OFFSETS into d_payload as
 * in cordahip_txcomp_batch): the components' leaf hashes straight from the
 * encoder's per-shape templates (no leaf bytes; new shapes are traced in the
 * same launch set, items without a template go through the direct encoder into
 * a SHA-256 sink, so there is no miss and no second pass) -> K4 Merkle roots ->
 * txid gather -> K1 verify -> K5 per-tx reduce, all on hip_stream. The ids of
 * cordahip_signed_txcomp_verify / cordahip_signed_tx_verify over the same
 * components' leaves; a rejected component makes its transaction
 * CORDAHIP_TX_BAD_COMPONENT and its signatures carry that status (as a failed
 * id does in every signed-tx path). group: as in cordahip_kryo_encode_device.
 * d_tx_item_off / d_tx_sig_off [ntx+1] (uint64) index d_items / the signatures
 * from 0; device memory is the caller's contract (not readable from the host).
 * n_items < 2^31 - 1. Replaces the same reference calls as
 * cordahip_txcomp_submit (SignedTransaction.kt:95-100, WireTransaction.kt:48,
 * MerkleTransaction.kt:16-18). */
int cordahip_signed_txcomp_verify_ed25519_device(cordahip_ctx* ctx, int device, const void* d_items,
                                                 uint64_t n_items, uint32_t group, const void* d_payload,
                                                 uint64_t payload_len, const void* d_tx_item_off, uint64_t ntx,
                                                 const void* d_tx_sig_off, const void* d_keys, const void* d_sigs,
                                                 uint64_t nsig, void* d_txid, void* d_tx_status, void* d_first_bad,
                                                 void* d_sig_status, void* hip_stream);

/* Device time (ms) of the calling thread's most recent *_device call on
 * `device`, from HIP events recorded around its launches on the stream it ran
 * on (waits for them); -1 if the thread made no such call. Each call gets its
 * own event pair from a per-device ring of 64, so concurrent callers on other
 * threads or streams do not disturb it -- up to 64 calls on the device in
 * between: after more, the slot has been reused and the result is -1. */
double cordahip_last_kernel_ms(cordahip_ctx* ctx, int device);

/* The in-process partition rule: shard `shard` of `nshards` over n lanes is
 * [*lo, *hi), contiguous, 64-aligned starts (whole verdict words), the last
 * shard possibly short or empty. Every multi-device host path uses it (per
 * scheme for generic batches; per transaction for tx batches, align 1). */
void cordahip_shard_range(uint64_t n, uint32_t nshards, uint32_t shard, uint64_t align, uint64_t* lo, uint64_t* hi);

#ifdef __cplusplus
}
#endif
#endif /* CORDAHIP_H */
