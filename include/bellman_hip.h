/*
 * bellman_hip.h -- C ABI of the MI355X-native Groth16 prover core.
 *
 * Drop-in boundary for the data-parallel hot path of doubiliu/bellman-mpc
 * (a fork of zkcrypto bellman 0.11.1).  Every entry point names the reference
 * interface it replaces (paths relative to bellman/src in the reference):
 *
 *   bh_multiexp            multiexp::multiexp            multiexp.rs:252-281
 *   bh_srs_upload          (Arc<Vec<G>>, usize) SourceBuilder / Parameters::read
 *                                                         multiexp.rs:45-86, groth16/mod.rs:292-400
 *   bh_fft / bh_ifft / bh_coset_fft / bh_icoset_fft /
 *   bh_distribute_powers / bh_divide_by_z_on_coset /
 *   bh_mul_assign / bh_sub_assign
 *                          EvaluationDomain methods      domain.rs:81-189
 *   bh_domain_size         EvaluationDomain::from_coeffs  domain.rs:47-79
 *   bh_evdom_*             EvaluationDomain with its coefficients resident in HBM
 *                                                         domain.rs:21-190
 *   bh_compute_h           the H block of create_proof   groth16/prover.rs:210-231
 *   bh_params_*            Parameters / ParameterSource  groth16/mod.rs:224-477
 *   bh_prove / bh_prove_witness
 *                          create_proof after synthesis   groth16/prover.rs:206-349
 *
 * Conventions
 *   - Plain pointers and sizes only; the caller owns every host buffer and the
 *     library never retains a caller pointer after a call returns -- except the inputs of
 *     bh_compute_h_scalars and bh_evdom_from_coeffs / bh_evdom_write, read asynchronously
 *     until the sync named there.
 *   - Fr vectors ("Montgomery") use the bls12_381 0.6 in-memory layout:
 *     4 little-endian u64 limbs of x * 2^256 mod r per element.
 *   - Exponents for bh_multiexp are Scalar::to_le_bits() words (canonical,
 *     4 LE u64 per scalar) unless BH_SCALARS_MONTGOMERY is given.  A canonical word
 *     >= r is taken mod r (the reference walks all 256 bits; k*P = (k mod r)*P in the
 *     prime-order group, so results agree).
 *   - Density maps are bitvec<u64, Lsb0> words: bit i of word i/64 is entry i.
 *   - Group elements use the zcash/bls12_381 encodings (big-endian, flag bits
 *     in byte 0): uncompressed 96 B (G1) / 192 B (G2), compressed 48/96 B.
 *   - Every function returns a bh_status; it never aborts across the FFI.
 *   - Process-wide side effect at load: GPU_MAX_HW_QUEUES is raised to 16 when it is
 *     unset or lower (HIP's default is 4; the prover keeps up to 12 streams busy and
 *     streams sharing a hardware queue serialise).  An explicitly set lower value is
 *     overridden too, with one line on stderr; BH_KEEP_HW_QUEUES=1 keeps the environment's
 *     value.  This only takes effect when the library loads before the first HIP call of
 *     the process.  Queue budget per context: DESIGN.md section 5.
 *   - bh_multiexp_submit jobs outlive nothing: destroying their context detaches every
 *     job not yet waited for, whose bh_multiexp_wait then returns BH_ERR_INVALID_ARGUMENT.
 */
#ifndef BELLMAN_HIP_H
#define BELLMAN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes mirror SynthesisError (lib.rs:355-364). */
typedef int bh_status;
#define BH_OK 0
#define BH_ERR_UNEXPECTED_IDENTITY 1     /* multiexp.rs:63-65, prover.rs:309-313 */
#define BH_ERR_UNEXPECTED_EOF 2          /* IoError(UnexpectedEof), multiexp.rs:55-61,74-80 */
#define BH_ERR_POLY_DEGREE_TOO_LARGE 3   /* domain.rs:57-59 */
#define BH_ERR_DENSITY_SIZE_MISMATCH 4   /* the reference panics (assert), multiexp.rs:277 */
#define BH_ERR_UNCONSTRAINED_VARIABLE 5  /* generator.rs:582-586 */
#define BH_ERR_INVALID_ARGUMENT 10
#define BH_ERR_INVALID_ENCODING 11       /* IoError(InvalidData) of Parameters::read */
#define BH_ERR_NOT_ON_CURVE 12          /* the checked decoders' InvalidData (mod.rs:292-400) */
#define BH_ERR_NOT_IN_SUBGROUP 14       /* same reference error: not torsion-free */
#define BH_ERR_OUT_OF_MEMORY 13
#define BH_ERR_SCRATCH_LIMIT 15          /* a kernel's spill scratch would exceed the device's limit (no reference counterpart) */
#define BH_ERR_HIP 100                   /* HIP runtime / device failure */

#define BH_G1 1
#define BH_G2 2

#define BH_SCALARS_CANONICAL 0
#define BH_SCALARS_MONTGOMERY 1

typedef struct bh_ctx bh_ctx;         /* one MI355X device + streams + workspaces (multicore.rs Worker) */
typedef struct bh_srs bh_srs;         /* device-resident affine base vector */
typedef struct bh_params bh_params;   /* device-resident Groth16 Parameters */
typedef struct bh_witness bh_witness; /* device-resident complete assignment */

const char* bh_status_string(bh_status s);
int bh_version(void);

/* ---- context (replaces multicore::Worker, multicore.rs:21-130) */
bh_status bh_ctx_create(int device, bh_ctx** out);
bh_status bh_ctx_destroy(bh_ctx* ctx);
/* Pre-allocate workspaces for MSMs up to max_msm_len and domains up to 2^max_log_domain,
 * so that later calls allocate nothing. */
bh_status bh_ctx_reserve(bh_ctx* ctx, size_t max_msm_len, uint32_t max_log_domain);
/* Force a window size for device MSMs (0 = automatic). Results never depend on it.
 * A forced window also disables the prover's window tables. */
bh_status bh_ctx_set_window(bh_ctx* ctx, int c);
/* Prover SRS window tables (default 1 = on): for each large query of the Parameters the
 * prover keeps T[i*W + w] = 2^(c*w) * P_i resident in HBM (built once per Parameters,
 * ~31 GB at 2^22 constraints on one GPU, 1/N of that per rank of an N-GPU run; skipped, with
 * a message on stderr, when HBM is short) so that all digit windows share one bucket set and
 * c can grow.  Results never depend on it. */
bh_status bh_ctx_set_tables(bh_ctx* ctx, int enable);

/* ---- bases (Source over Arc<Vec<G1Affine|G2Affine>>) */
bh_status bh_srs_upload(bh_ctx* ctx, int group, const uint8_t* uncompressed_be, size_t n, int checked,
                        bh_srs** out);
bh_status bh_srs_free(bh_srs* srs);
size_t bh_srs_len(const bh_srs* srs);
/* read back base i as uncompressed bytes (96/192 B) */
bh_status bh_srs_get(const bh_srs* srs, size_t i, uint8_t* out);

/* ---- multiexp::multiexp.  density_words == NULL means FullDensity.  out: uncompressed
 * encoding of the projective result normalised to affine (96 B for G1, 192 B for G2). */
bh_status bh_multiexp(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint64_t* density_words,
                      size_t density_len, const uint64_t* exponents, size_t n, int scalar_format, uint8_t* out);

/* ---- asynchronous multiexp: multiexp::multiexp returns a Waiter (multiexp.rs:252-281,
 * multicore.rs:94-110) and create_proof keeps eight in flight (prover.rs:233-307).  submit
 * enqueues the multiexp on a stream and workspace of its own and returns without waiting for
 * the device (the exponents and density words are read before it returns); wait blocks on
 * the job's event, writes the result like bh_multiexp and frees the job.  EOF / identity
 * errors of the Source are reported by wait, as the reference reports them from wait().
 * Thread-safe: any number of jobs per context, submitted and waited from any threads. */
typedef struct bh_job bh_job;
bh_status bh_multiexp_submit(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint64_t* density_words,
                             size_t density_len, const uint64_t* exponents, size_t n, int scalar_format,
                             bh_job** out);
bh_status bh_multiexp_wait(bh_job* job, uint8_t* out);

/* ---- the same seam on device-resident data.  create_proof clones one Arc<Vec<Fr::Repr>> per
 * assignment into several multiexps (prover.rs:233-307) and builds h into another
 * (prover.rs:227-231): a bh_scalars is that Arc on the device -- uploaded once (canonical or
 * Montgomery words, like bh_multiexp), or produced by bh_compute_h_scalars -- and any number of
 * multiexps read it.  bh_compute_h_scalars returns at once: a host thread uploads a, b, c and
 * enqueues the H passes, and multiexps submitted on h meanwhile are enqueued by that thread
 * behind them, so a caller can submit in create_proof's own order (h first) without waiting.  That
 * deferral is for submits on the producing context; a submit on another context of the device
 * first waits (on the host) until the producer has enqueued H, then enqueues normally.  Freeing the
 * handle is allowed while multiexps on it are in flight (they keep the device vector until their
 * wait). */
typedef struct bh_scalars bh_scalars;
bh_status bh_scalars_upload(bh_ctx* ctx, const uint64_t* exponents, size_t n, int scalar_format, bh_scalars** out);
bh_status bh_compute_h_scalars(bh_ctx* ctx, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                               size_t num_constraints, bh_scalars** h_out);
size_t bh_scalars_len(const bh_scalars* s);
bh_status bh_scalars_free(bh_scalars* s);
/* bh_compute_h_scalars reads a, b, c from a host thread of its own: they stay borrowed until this
 * returns (or a multiexp on the vector has been waited, or the vector is freed).  Returns the
 * H block's status (also reported by every multiexp waited on it). */
bh_status bh_scalars_sync(bh_scalars* s);
/* Profile of bh_compute_h_scalars' producer (waits like bh_scalars_sync), ms since the call:
 * [0..3) the copies of a, b, c enqueued, [3] the H passes enqueued, [4] the multiexps deferred
 * behind it enqueued, [5] how many were deferred.  A vector from bh_scalars_upload reports -1s. */
bh_status bh_scalars_stamps(bh_scalars* s, double out[6]);
bh_status bh_multiexp_submit_scalars(bh_ctx* ctx, const bh_srs* bases, size_t base_offset,
                                     const uint64_t* density_words, size_t density_len, const bh_scalars* exps,
                                     bh_job** out);

/* ---- EvaluationDomain.  Arrays hold 2^log_m Montgomery Fr (4 u64 each), in place. */
bh_status bh_domain_size(size_t len, size_t* m, uint32_t* log_m);
bh_status bh_fft(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m);
bh_status bh_ifft(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m);
bh_status bh_coset_fft(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m);
bh_status bh_icoset_fft(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m);
bh_status bh_distribute_powers(bh_ctx* ctx, uint64_t* coeffs, size_t len, const uint64_t g_mont[4]);
bh_status bh_divide_by_z_on_coset(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m);
bh_status bh_mul_assign(bh_ctx* ctx, uint64_t* a, const uint64_t* b, size_t len);
bh_status bh_sub_assign(bh_ctx* ctx, uint64_t* a, const uint64_t* b, size_t len);
/* ---- EvaluationDomain with its coefficients resident in HBM (domain.rs:21-190).  The
 * reference keeps `coeffs` private behind AsRef/AsMut/into_coeffs (domain.rs:21-45), so a
 * binding can hold them on the device from from_coeffs to into_coeffs: each method below is
 * an enqueue on the context's stream, and only bh_evdom_read / bh_evdom_into_scalars move
 * data back.  A handle belongs to its context (free it before the context) and is used by one
 * thread at a time (the reference's &mut self); different handles of one context may be used
 * from different threads.
 *   bh_evdom_from_coeffs   EvaluationDomain::from_coeffs   domain.rs:47-79 (zero-padded to 2^exp;
 *                          BH_ERR_POLY_DEGREE_TOO_LARGE past 2^31).  `coeffs` (len Montgomery Fr, 4 u64
 *                          each) is read asynchronously by the context's upload thread, in call
 *                          order: it stays borrowed until bh_evdom_sync (or read / into_scalars /
 *                          free) returns
 *   bh_evdom_fft / _ifft / _coset_fft / _icoset_fft      domain.rs:81-127
 *   bh_evdom_distribute_powers                           domain.rs:101-113
 *   bh_evdom_divide_by_z_on_coset                        domain.rs:139-151
 *   bh_evdom_mul_assign / _sub_assign                    domain.rs:153-189 (lengths must agree:
 *                          BH_ERR_INVALID_ARGUMENT, where the reference asserts)
 *   bh_evdom_read          as_ref / into_coeffs: the first len (<= m) coefficients, Montgomery
 *   bh_evdom_write         as_mut written back: replaces the coefficients by len (<= m) values,
 *                          zero-padded (asynchronous like from_coeffs)
 *   bh_evdom_into_scalars  prover.rs:226-231: the first len (<= m) coefficients as canonical
 *                          scalars (to_le_bits) in a device vector for bh_multiexp_submit_scalars,
 *                          without leaving the device; consumes the domain (later calls fail with
 *                          BH_ERR_INVALID_ARGUMENT, free still required) */
typedef struct bh_evdom bh_evdom;
bh_status bh_evdom_from_coeffs(bh_ctx* ctx, const uint64_t* coeffs, size_t len, bh_evdom** out);
bh_status bh_evdom_size(const bh_evdom* d, size_t* m, uint32_t* log_m);
bh_status bh_evdom_fft(bh_evdom* d);
bh_status bh_evdom_ifft(bh_evdom* d);
bh_status bh_evdom_coset_fft(bh_evdom* d);
bh_status bh_evdom_icoset_fft(bh_evdom* d);
bh_status bh_evdom_distribute_powers(bh_evdom* d, const uint64_t g_mont[4]);
bh_status bh_evdom_divide_by_z_on_coset(bh_evdom* d);
bh_status bh_evdom_mul_assign(bh_evdom* d, bh_evdom* other);
bh_status bh_evdom_sub_assign(bh_evdom* d, bh_evdom* other);
bh_status bh_evdom_read(bh_evdom* d, uint64_t* out, size_t len);
bh_status bh_evdom_write(bh_evdom* d, const uint64_t* coeffs, size_t len);
bh_status bh_evdom_into_scalars(bh_evdom* d, size_t len, bh_scalars** out);
bh_status bh_evdom_sync(bh_evdom* d);
bh_status bh_evdom_free(bh_evdom* d);

/* H block of create_proof: a, b, c hold num_constraints evaluations each (padded to m
 * internally); h_out receives m-1 Montgomery coefficients; *h_len = m-1. */
bh_status bh_compute_h(bh_ctx* ctx, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                       size_t num_constraints, uint64_t* h_out, size_t* h_len);

/* ---- Parameters (groth16/mod.rs:224-477) */
/* Parameters::read format (VerifyingKey::write then u32-BE length-prefixed h, l, a, b_g1, b_g2). */
bh_status bh_params_load(bh_ctx* ctx, const uint8_t* bytes, size_t len, int checked, bh_params** out);
bh_status bh_params_free(bh_params* p);
/* sizes: [h, l, a, b_g1, b_g2, ic] */
bh_status bh_params_sizes(const bh_params* p, size_t out[6]);
/* ParameterSource::get_h / get_l / get_a / get_b_g1 / get_b_g2 (groth16/mod.rs:414-477): the
 * Parameters' own base vector as a bh_srs, borrowed (valid while p lives; never bh_srs_free it).
 * Multiexps over it (bh_multiexp_submit*) use the window tables bh_params_prepare built, as
 * bh_prove does: the seam then runs at the prover's per-multiexp speed. */
#define BH_VEC_H 0
#define BH_VEC_L 1
#define BH_VEC_A 2
#define BH_VEC_B_G1 3
#define BH_VEC_B_G2 4
bh_status bh_params_vector(const bh_params* p, int which, const bh_srs** out);

/* ---- prover (create_proof after synthesis, prover.rs:206-349) */
/* a,b,c: num_constraints Montgomery Fr (ProvingAssignment a/b/c incl. the input constraints);
 * assignments Montgomery; densities: bit words (a_aux: num_aux bits, b_input: num_inputs bits,
 * b_aux: num_aux bits); r, s canonical (4 LE u64).  proof_out: Proof::write, 192 B. */
bh_status bh_prove(bh_ctx* ctx, const bh_params* params, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                   size_t num_constraints, const uint64_t* input_assignment, size_t num_inputs,
                   const uint64_t* aux_assignment, size_t num_aux, const uint64_t* a_aux_density,
                   const uint64_t* b_input_density, const uint64_t* b_aux_density, const uint64_t r[4],
                   const uint64_t s[4], uint8_t proof_out[192]);
/* Same, split into an upload (witness becomes device-resident) and the proof proper. */
bh_status bh_witness_upload(bh_ctx* ctx, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                            size_t num_constraints, const uint64_t* input_assignment, size_t num_inputs,
                            const uint64_t* aux_assignment, size_t num_aux, const uint64_t* a_aux_density,
                            const uint64_t* b_input_density, const uint64_t* b_aux_density, bh_witness** out);
bh_status bh_witness_free(bh_witness* w);
/* Build now (instead of inside the first proof) the window tables that proofs of witnesses
 * shaped like w, split over nshards GPUs, will use.  Optional. */
bh_status bh_params_prepare(bh_ctx* ctx, bh_params* params, const bh_witness* w, size_t nshards);
/* The same for ONE shard: only the slices of the query vectors that shard `shard` of
 * `nshards` consumes (and, with distributed_h, its gathered share of the h vector), so that
 * a rank of a multi-GPU run holds and builds 1/nshards of the tables.  Optional. */
bh_status bh_params_prepare_shard(bh_ctx* ctx, bh_params* params, const bh_witness* w, size_t shard, size_t nshards,
                                  int distributed_h);
bh_status bh_prove_witness(bh_ctx* ctx, const bh_params* params, const bh_witness* w, const uint64_t r[4],
                           const uint64_t s[4], uint8_t proof_out[192]);

/* Throughput mode (BASELINE.json configs[4], "C5"): k independent proofs of witnesses sharing
 * one Parameters (the reference's Worker::compute fan-out, multicore.rs:33-76, r and s fixed,
 * prover.rs:158-173), every window table built once up front.  lanes (0 = default, 2): with 1
 * the proofs run back to back on ctx; with L >= 2, L host threads drive L lane contexts that
 * borrow ctx's streams (no hardware queue more) and take turns in proof order, proof i+1 being
 * enqueued as soon as proof i's device work is -- its density maps, sorts and H then run beside
 * proof i's last reduction tail and host combine.  proofs_out: k * 192 bytes, proof i ==
 * bh_prove_witness(ws[i]).  Across GPUs the batch is split by the caller (one process per GPU,
 * no collective). */
bh_status bh_prove_batch(bh_ctx* ctx, const bh_params* params, const bh_witness* const* ws, size_t k,
                         const uint64_t r[4], const uint64_t s[4], int lanes, uint8_t* proofs_out);

/* ---- multi-GPU: every multiexp sharded by scalar range (shard k of N covers
 * [k*n/N, (k+1)*n/N) of each query); partial_out = 8 uncompressed points
 * [h, l, a_inputs, a_aux, b_g1_inputs, b_g1_aux] (G1, 96 B) + [b_g2_inputs, b_g2_aux]
 * (G2, 192 B) = 960 B.  The all-gathered records are summed and assembled on the
 * host by bh_proof_from_partials (prover.rs:315-349), which needs only the
 * VerifyingKey::write bytes (bh_vk_write). */
#define BH_PARTIAL_BYTES 960
bh_status bh_shard_range(size_t n, size_t shard, size_t nshards, size_t* lo, size_t* hi);
bh_status bh_prove_witness_partial(bh_ctx* ctx, const bh_params* params, const bh_witness* w, size_t shard,
                                   size_t nshards, uint8_t partial_out[960]);
bh_status bh_vk_write(const bh_params* p, uint8_t* out, size_t cap, size_t* written);

/* ---- verification (host only, no device needed): verify_proof (verifier.rs:11-62) and the batch
 * verifier (verifier/batch.rs:95-169) over a BLS12-381 pairing.  vk: VerifyingKey::write bytes (the
 * head of Parameters::write, or bh_vk_write); proof: Proof::write bytes (192, decoded like Proof::read:
 * compressed, torsion-checked, identity rejected); public inputs: num_inputs canonical Fr, 4 LE u64
 * each, without the implicit ONE.  *valid = 1 iff the proof(s) verify; the status is non-zero only for
 * malformed data (num_inputs + 1 != ic length: BH_ERR_INVALID_ARGUMENT, the reference's
 * VerificationError::InvalidVerifyingKey).  Batch: k proofs, inputs k * num_inputs * 4 words, and the
 * caller's random nonzero scalars z (k * 4 canonical words; the reference draws them from a CryptoRng). */
bh_status bh_verify_proof(const uint8_t* vk, size_t vk_len, const uint8_t* proof, const uint64_t* inputs,
                          size_t num_inputs, int* valid);
bh_status bh_verify_batch(const uint8_t* vk, size_t vk_len, const uint8_t* proofs, const uint64_t* inputs,
                          size_t num_inputs, size_t k, const uint64_t* z, int* valid);
bh_status bh_proof_from_partials(const uint8_t* vk_bytes, size_t vk_len, const uint8_t* partials, size_t nshards,
                                 const uint64_t r[4], const uint64_t s[4], uint8_t proof_out[192]);

/* RCCL exchange (one communicator per rank/device; unique id shared out of band) */
typedef struct bh_comm bh_comm;
bh_status bh_comm_unique_id(uint8_t out[128]);
bh_status bh_comm_init(bh_ctx* ctx, const uint8_t id[128], int nranks, int rank, bh_comm** out);
/* all ranks' records, rank order: all_out holds nranks * BH_PARTIAL_BYTES bytes */
bh_status bh_comm_allgather_partials(bh_comm* c, const uint8_t* partial, uint8_t* all_out);
bh_status bh_comm_destroy(bh_comm* c);
/* every rank's nbytes-byte host record, rank order, into all_out (nranks * nbytes) */
bh_status bh_comm_allgather(bh_comm* c, const uint8_t* in, size_t nbytes, uint8_t* all_out);
/* max over ranks of *inout (in place, every rank); returns once every rank has called it,
 * so it is also the barrier around a timed region */
bh_status bh_comm_allreduce_max(bh_comm* c, double* inout);
/* what RCCL reports for the communicator: out = {rank count, this rank, HIP device id} */
bh_status bh_comm_info(const bh_comm* c, int out[3]);
/* This rank's partial record (rank/nranks from the communicator).  For nranks a power of two
 * in [2, 16] and m >= 2*nranks^2 the H block is distributed instead
 * of replicated: every NTT is a local m/nranks-point NTT plus one ncclSend/ncclRecv
 * all-to-all, three all-to-alls per proof, and this rank's h multiexp covers exactly the h
 * coefficients it ends with (a strided set, not the range of bh_shard_range).  Otherwise
 * identical to bh_prove_witness_partial(ctx, params, w, rank, nranks, ...). */
bh_status bh_prove_witness_partial_comm(bh_ctx* ctx, const bh_params* params, const bh_witness* w, bh_comm* comm,
                                        uint8_t partial_out[960]);
/* All nshards partial records computed on this one device by nshards virtual ranks: each a
 * context and a host thread of its own running the per-rank code of
 * bh_prove_witness_partial_comm, with device copies in place of the RCCL all-to-alls
 * (rehearsal and tests of the multi-GPU algorithm).  partials_out: nshards * BH_PARTIAL_BYTES. */
bh_status bh_prove_witness_partials_local(bh_ctx* ctx, const bh_params* params, const bh_witness* w,
                                          size_t nshards, uint8_t* partials_out);
/* The same with caller-provided ranks of one device: ctxs[k] and params[k] are rank k's context
 * and Parameters (e.g. loaded per rank and prepared with bh_params_prepare_shard, exactly as
 * the processes of a multi-GPU run hold them); the witness is shared. */
bh_status bh_prove_witness_partials_ranks(bh_ctx* const* ctxs, const bh_params* const* params, const bh_witness* w,
                                          size_t nranks, uint8_t* partials_out);
/* Rehearsal of rank `rank` of an nranks-GPU run on this one device: exactly that rank's
 * device work (its shards, the distributed H block when it applies) with each all-to-all
 * moving only the rank's own chunks; *ms = host wall time of the rank's proof.  The partial
 * sums are discarded (the data crossing ranks is missing): for timing and profiling only. */
bh_status bh_rehearse_rank(bh_ctx* ctx, const bh_params* params, const bh_witness* w, size_t rank, size_t nranks,
                           double* ms);
bh_status bh_ctx_synchronize(bh_ctx* ctx);
int bh_device_count(void);

/* ---- synthetic workload: MiMC chain (mimc_mod.rs:40-130 with R rounds, seeded constants),
 * synthesized natively (witness) and its CRS generated on the device with the classic
 * algorithm (generator.rs:310-572) from the given toxic waste (canonical u64 each). */
bh_status bh_chain_witness(bh_ctx* ctx, size_t rounds, uint64_t seed, bh_witness** out);
/* Same circuit (constants from seed), preimage (xl, xr) from preimage_seed: distinct
 * witnesses for one set of Parameters (BASELINE.json configs[4], "C5").
 * bh_chain_witness(seed) == bh_chain_witness_preimage(seed, seed + 1). */
bh_status bh_chain_witness_preimage(bh_ctx* ctx, size_t rounds, uint64_t seed, uint64_t preimage_seed,
                                    bh_witness** out);
/* The chain's ProvingAssignment on the host, in exactly the layouts bh_prove takes (the
 * drop-in path a Rust caller uses after synthesis): sizes = {constraints, inputs, aux};
 * a, b, c: constraints x 4 u64 Montgomery; inputs/aux Montgomery; density bit words. */
bh_status bh_chain_sizes(size_t rounds, size_t out[3]);
bh_status bh_chain_assignment(size_t rounds, uint64_t seed, uint64_t preimage_seed, uint64_t* a, uint64_t* b,
                              uint64_t* c, uint64_t* inputs, uint64_t* aux, uint64_t* a_aux_density,
                              uint64_t* b_input_density, uint64_t* b_aux_density);
bh_status bh_chain_params(bh_ctx* ctx, size_t rounds, uint64_t seed, uint64_t alpha, uint64_t beta, uint64_t gamma,
                          uint64_t delta, uint64_t tau, bh_params** out);
/* Parameters::write of device-resident params (for parity tests; host copy). */
bh_status bh_params_write(const bh_params* p, uint8_t* out, size_t cap, size_t* written);

/* ---- profile of the last bh_prove_witness[_partial] (device events):
 * [0] host wall ms, [1] H pipeline ms, [2] G1 accumulation ms (sum over launches),
 * [3] G1 accumulation launches, [4] G1 (base, scalar) pairs, [5] G2 accumulation ms,
 * [6] G2 launches, [7] G2 pairs, [8] G1 mixed additions, [9] G2 mixed additions */
bh_status bh_last_timings(const bh_ctx* ctx, double out[10]);
/* bh_last_timings' fields followed by [10] large multiexps that used a window table,
 * [11] large multiexps (those a table would serve), [12] bytes of the window tables the proof
 * read (each distinct table once: for a shard, its own slices); after a bh_prove from host
 * buffers, [13] ms from the call's start until inputs + aux had landed on the device, [14..16]
 * until a, b, c had, [17] until the H block was done; after bh_fft / bh_ifft / bh_coset_fft /
 * bh_icoset_fft, [18] upload, [19] transform, [20] download ms of the last call; after a proof,
 * [21] / [22] the wall time (ms) during which at least one G1 / G2 bucket accumulation ran (the
 * union of their launches; [2] and [5] sum the launches, which can overlap); n entries are
 * written (missing ones 0). */
bh_status bh_last_stats(const bh_ctx* ctx, double* out, size_t n);

/* ---- scratch budget (no reference counterpart: a guard the device needs).  A spilling kernel's
 * scratch is provisioned per hardware queue for the waves it can have in flight, out of one
 * device-wide amount; exceeding it aborts inside the runtime (HSA_STATUS_ERROR_OUT_OF_RESOURCES).
 * The library checks its kernels (private segment per lane x 64 x resident waves, times the
 * queues a context runs them on) against the device limit before every proof and multiexp, which
 * return BH_ERR_SCRATCH_LIMIT instead.  out[0..n): [0] device scratch limit (bytes, shared by all
 * queues; 0 unknown), [1] current per-queue threshold, [2] worst private segment (bytes/lane),
 * [3] its per-queue need at the scratch-slot bound (32 waves per CU), [4] queues counted, [5] the
 * context's total need, [6] fits (1/0), [7] kernels checked, [8] the worst kernel's per-queue need
 * at its occupancy, [9] live contexts on the device (refreshed on every call); worst_kernel
 * (optional, cap bytes): that kernel's name.  [6] decides for ONE context's queues: a caller that
 * runs several contexts' proofs at once on one device must budget [5] x [9] itself (batch lanes
 * borrow their primary's streams; the one-device rehearsal's ranks prove one after another). */
bh_status bh_scratch_report(bh_ctx* ctx, uint64_t* out, size_t n, char* worst_kernel, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* BELLMAN_HIP_H */
