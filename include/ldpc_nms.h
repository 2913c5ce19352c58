/*
 * ldpc_nms.h — C ABI of the MI355X neural min-sum (NMS / quantized NMS) LDPC decoder.
 *
 * The reference (ghy1228/LDPC_Error_Floor) has no FFI: its decoder is a TF1 graph built by
 * build_neural_network (Main_Functions.py:157-385) and executed through
 *     sess.run(fetches=net_dict["ya_output_all"] [, net_dict["lossa"]],
 *              feed_dict={xa: X[B,N,z], ya: Y, etha: e, learn_rate: 0})
 * (Print_Functions.py:147-151).  Each entry point below replaces one piece of that:
 *
 *   ldpc_graph_create   <- init_parameter + init_connecting_matrix (Main_Functions.py:8-150)
 *   ldpc_weights_set    <- weight_init's var_{i}_{t} (Main_Functions.py:387-439), already
 *                          expanded per iteration by the sharing rules (:167-174, :266-304)
 *   ldpc_ctx_create     <- the placeholders' fixed batch size (main_Base.py:122-127)
 *   ldpc_decode         <- sess.run of the T unrolled iterations; app_all == ya_output_all,
 *                          counters == calc_ber_fer (Print_Functions.py:100-118) on device
 *
 * Conventions: LLRs are log(p1/p0) (Print_Functions.py:45-46), bit index j*z+g, proto edges
 * in row-major order E(C).  All device pointers are owned by the caller (e.g. torch
 * tensors); the library owns graph tables, weights and per-context scratch.  Every call
 * returns LDPC_OK (0) or a negative status; no exception crosses the boundary.  A context
 * must be used by one host thread / stream at a time; there is no global mutable state.
 */
#ifndef LDPC_NMS_H
#define LDPC_NMS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_NMS_ABI_VERSION 3     /* 2: ldpc_decode_outputs.iter_wrong, ldpc_ctx_last_kernel;
                                      3: ldpc_decode_params.outputs_size */

typedef struct ldpc_graph ldpc_graph;
typedef struct ldpc_ctx ldpc_ctx;

enum ldpc_status {
    LDPC_OK = 0,
    LDPC_ERR_ARG = -1,          /* bad argument (null pointer, size, unsupported mode) */
    LDPC_ERR_HIP = -2,          /* a HIP runtime call or kernel launch failed */
    LDPC_ERR_OOM = -3,          /* device allocation failed */
    LDPC_ERR_STATE = -4,        /* weights not set / B or T above the context limits */
    LDPC_ERR_UNSUPPORTED = -5   /* valid request this build cannot serve */
};

enum ldpc_decoding_type {       /* decoding_type of main_Base.py:27 */
    LDPC_DEC_SP = 0,            /* sum-product: tanh / atanh check update (flood kernel) */
    LDPC_DEC_MS = 1,            /* min-sum fp32, messages clipped to +-clip_llr */
    LDPC_DEC_QMS = 2,           /* quantized min-sum on the q_bit grid */
    LDPC_DEC_MS_NONUDGE = 3     /* min-sum without the 0 -> 1e-4 nudge */
};

enum ldpc_kernel {
    LDPC_KERNEL_AUTO = 0,       /* fused when supported, else flooding */
    LDPC_KERNEL_FLOOD = 1,      /* two edge-parallel kernels per iteration, state in HBM */
    LDPC_KERNEL_FUSED = 2       /* all T iterations in one launch, state in LDS/registers */
};

typedef struct ldpc_decode_params {
    int32_t T;                  /* iterations (training_iter_end), 1 <= T <= T_max */
    int32_t decoding_type;      /* ldpc_decoding_type */
    int32_t q_bit;              /* 6, 5, -5, 4 or 3 (QMS only) */
    int32_t target_bits;        /* Nt*z: width of app_all and of the FER/BER bit range */
    float clip_llr;             /* clip_LLR (20.0 in the reference) */
    int32_t kernel;             /* ldpc_kernel */
    int32_t outputs_size;       /* sizeof(ldpc_decode_outputs) the caller was built with: 0 = the
                                   ABI-1 struct (five pointers, no iter_wrong; ABI-1 callers zeroed
                                   this word as reserved), sizeof(ldpc_decode_outputs) = this
                                   header's struct; any other value -> LDPC_ERR_ARG.  The library
                                   never reads past the size the caller declares.  An ABI-2
                                   binary (iter_wrong set, this word zeroed as reserved[0]) is
                                   read as ABI 1 and gets no iter_wrong: ABI-2 callers must be
                                   rebuilt against this header, and a caller relying on
                                   iter_wrong checks ldpc_abi_version() >= 3 first. */
    int32_t reserved;
} ldpc_decode_params;

typedef struct ldpc_decode_outputs {
    float* app_all;             /* [T][B][target_bits] f32 (== ya_output_all) or NULL */
    uint32_t* hard_bits;        /* [T][B][ceil(N*z/32)] bit v%32 of word v/32, or NULL */
    uint32_t* synd_bits;        /* [T][B][ceil(M*z/32)] syndrome of hard_bits[t], or NULL */
    int64_t* counters;          /* [4] += {bit errors @T-1, frames wrong @T-1,
                                   frames wrong at every t, 2*loss (loss_type 2, etha 0)}
                                   for the all-zero codeword; or NULL */
    uint8_t* frame_flags;       /* [B] bit0 wrong at every t (uncor), bit1 wrong @T-1; or NULL */
    uint32_t* iter_wrong;       /* [T][ceil(B/32)]: bit b%32 of word (t, b/32) = frame b has a hard
                                   decision 1 among the target bits at iteration t (the per-iteration
                                   frame error of calc_ber_fer, Print_Functions.py:100-118; the
                                   all-zero codeword), bits past B zero; or NULL.  Every kernel
                                   serves it, the counters-only ones included.  Read only when
                                   ldpc_decode_params.outputs_size declares it (ABI 3). */
} ldpc_decode_outputs;

int ldpc_abi_version(void);
const char* ldpc_status_string(int status);

/* proto: host [M][N] row-major, -1 = no edge, else cyclic shift (taken mod z). */
int ldpc_graph_create(const int32_t* proto, int32_t M, int32_t N, int32_t z, int32_t device,
                      ldpc_graph** out);
int ldpc_graph_destroy(ldpc_graph* g);
/* dims[8] = {M, N, z, E, n_checks, n_vars, n_edges, max_check_degree} */
int ldpc_graph_query(const ldpc_graph* g, int32_t* dims);

/* Host tables, copied to the device: alpha [T][E] (E(C) order), alpha_ucn [T][E] or NULL
   (UCN weighting off), beta [T][N]. */
int ldpc_weights_set(ldpc_graph* g, int32_t T, const float* alpha, const float* alpha_ucn,
                     const float* beta);

int ldpc_ctx_create(ldpc_graph* g, int64_t B_max, int32_t T_max, ldpc_ctx** out);
int ldpc_ctx_destroy(ldpc_ctx* c);

/* llr_dev: device [B][N*z] f32 (natural bit order, log p1/p0).  stream: hipStream_t (NULL =
   default stream).  Asynchronous: returns after enqueueing on the stream. */
int ldpc_decode(ldpc_ctx* c, const float* llr_dev, int64_t B, const ldpc_decode_params* p,
                const ldpc_decode_outputs* o, void* stream);

/* Bytes of HBM traffic per codeword the selected kernel is designed to move (for the
   roofline report), and a short kernel name.  Returns 0 if unsupported. */
int ldpc_kernel_info(const ldpc_ctx* c, const ldpc_decode_params* p, int64_t* bytes_per_cw,
                     char* name, int32_t name_len);

/* Name of the kernel that served the last successful ldpc_decode / ldpc_decode_awgn on this
   context (empty before the first).  Which kernel runs depends on the requested outputs: APP
   exports run v5 or flood, counters / frame flags / iter_wrong / hard_bits / synd_bits of the
   QMS grids the bit-sliced kernels ("bsl[...]", "bsc[...]"), whose hard-bit export is a
   separate build of the same kernel that also stores each iteration's hard decisions. */
int ldpc_ctx_last_kernel(const ldpc_ctx* c, char* name, int32_t name_len);

/* On-GPU AWGN channel for the all-zero codeword (create_mix_epoch, Print_Functions.py:29-72):
   writes llr_dev [B][n_vars] f32 = Q(2(sigma*n - 1)/sigma^2) with punctured (1-based bits
   punct_start..punct_end, 0 = none) -> 0 and shortened -> -clip_llr.  Counter-based Philox
   streams indexed by (seed, offset + b, element): shards generated with their global codeword
   offset reproduce the single-GPU stream.  QMS: the quantized level is sampled exactly from
   its distribution (64-bit CDF thresholds computed in float64, one Philox per 4 codewords of a
   variable); float modes: Box-Muller with a 53-bit uniform under the logarithm (tails to ~8.6
   sigma).  See csrc/ldpc_awgn.h. */
int ldpc_channel_awgn(float* llr_dev, int64_t B, int32_t n_vars, double sigma, uint64_t seed,
                      int64_t offset, int32_t decoding_type, int32_t q_bit, int32_t punct_start,
                      int32_t punct_end, int32_t short_start, int32_t short_end, float clip_llr,
                      void* stream);

/* In-decoder channel for throughput sweeps (SURVEY §8 f rank 1): the LLRs of the B codewords
   come from the same generator as ldpc_channel_awgn (same seed, global codeword offset,
   puncture/shorten) and never cross HBM as floats: APP exports generate them in the fused v5
   kernel's prologue; counters-only QMS decodes of the bit-sliced kernels take a byte channel
   (one byte per LLR, already in the layout their prologue packs into bit planes); flood and the
   float-mode kernel generate float LLRs into a context buffer first.  The result is identical to
   ldpc_channel_awgn followed by ldpc_decode.  Replaces create_mix_epoch + sess.run in the
   compute_results loop (Print_Functions.py:29-72, :130-165). */
typedef struct ldpc_channel_params {
    double sigma;                 /* noise standard deviation (SNR -> sigma: init_parameter) */
    uint64_t seed;
    int64_t offset;               /* global index of the batch's first codeword */
    int32_t punct_start, punct_end, short_start, short_end;   /* 1-based, 0 = none */
    int32_t reserved[4];
} ldpc_channel_params;

int ldpc_decode_awgn(ldpc_ctx* ctx, int64_t B, const ldpc_decode_params* params,
                     const ldpc_channel_params* channel, const ldpc_decode_outputs* outputs,
                     void* stream);

/* Whether ldpc_decode_awgn with these parameters generates the channel inside the decoding
   kernel (the v5 prologue for APP exports, the bit-sliced kernels' prologue for counters-only QMS
   decodes): 1, else 0 (the channel kernel writes float LLRs to the context's buffer first), or a
   negative status.  has_short: the channel has shortened bits; app: an APP export is asked for.
   The decision ldpc_decode_awgn itself takes; a decode it served in-kernel also reports its
   kernel through ldpc_ctx_last_kernel with the suffix "+gen". */
int ldpc_awgn_in_kernel(const ldpc_ctx* ctx, const ldpc_decode_params* params, int32_t has_short,
                        int32_t app);

/* The LLR rows ldpc_channel_awgn(B, ..., offset) would write at batch rows idx_dev[0..n) (each
   index < B, any order), into rows_dev[n][n_vars]: the same values bit for bit, generated for
   those codewords only -- the uncorrected-word sweep regenerates the few failing frames' rows
   after a decode whose channel was generated inside the kernel (ldpc_decode_awgn). */
int ldpc_channel_awgn_rows(float* rows_dev, const int64_t* idx_dev, int64_t n, int32_t n_vars,
                           double sigma, uint64_t seed, int64_t offset, int32_t decoding_type,
                           int32_t q_bit, int32_t punct_start, int32_t punct_end,
                           int32_t short_start, int32_t short_end, float clip_llr, void* stream);

/* Uncorrected-frame collection for the on-device sweep (replaces the host selection in
   compute_results -> write_uncor_file, Print_Functions.py:155-156 and :120-126).
   Writes the indices b < B with (frame_flags[b] & mask) == want into idx_dev[0..cap) (order
   within the batch is not preserved: sort the few indices on the host) and the number of
   matches (which may exceed cap) into *count_dev (zeroed by the call).  With the decoder's
   frame_flags, mask = want = 1 selects the frames wrong at every iteration (uncor_flag). */
int ldpc_collect_frames(const uint8_t* flags_dev, int64_t B, uint32_t mask, uint32_t want,
                        int64_t* idx_dev, int64_t cap, int64_t* count_dev, void* stream);

/* dst[r][:] = src[idx[r]][:] for r < n (n <= 65535 per call): the LLR rows of the collected
   frames, on the device, before the copy to the host. */
int ldpc_gather_rows(const float* src_dev, int64_t n_cols, const int64_t* idx_dev, int64_t n,
                     float* dst_dev, void* stream);

/* Host: the text of write_uncor_file's rows (Print_Functions.py:120-126, np.savetxt with
   fmt "%.1f", tab-delimited) for n float32 LLR rows of n_cols values: "0.0\t0.0\t0.0\t" then
   the negated LLRs, byte-identical to np.savetxt's output.  cap must be at least
   n * LDPC_UNCOR_ROW_BOUND(n_cols); *len = the bytes written. */
#define LDPC_UNCOR_ROW_BOUND(n_cols) (13 + 48 * (int64_t)(n_cols))
int ldpc_format_uncor_rows(const float* rows, int64_t n, int64_t n_cols, char* out, int64_t cap,
                           int64_t* len);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_NMS_H */
