// kfamd_kernels.h — C ABI of the hand-written CDNA4 (gfx950) kernel library.
//
// This library is the MI355X compute path of the framework (SURVEY.md §2.7.2, K1–K3):
//   K1  bf16 GEMM on MFMA (v_mfma_f32_16x16x32_bf16), LDS-tiled, global_load_lds staging
//   K2  LayerNorm / RMSNorm forward+backward (bf16 I/O, fp32 statistics)
//   K3  one-shot peer all-reduce for small messages (allreduce_oneshot.hip); large messages
//       go to RCCL (native/readiness, kubeflow_rm_amd.parallel)
//
// It is consumed three ways, all in-tree:
//   * Python (kubeflow_rm_amd.ops) through ctypes — one HIP runtime shared with torch;
//   * the native in-pod readiness op (native/readiness) linked directly;
//   * the bench harness (bench.py) through the Python ops.
//
// Every launcher is asynchronous on the given stream and never allocates, syncs or copies,
// so callers may capture it into a hipGraph (cdna_hip_programming.md §6 G9).
// Return value: 0 on success, otherwise a negative kfamd_status code (shape/alignment
// contract violated) or a positive hipError_t from the launch.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum kfamd_status {
  KFAMD_OK = 0,
  KFAMD_EINVAL = -1,     // bad shape / null pointer
  KFAMD_EALIGN = -2,     // pointer or leading dimension not 16-byte aligned for the fast path
};

// Epilogue activation codes for the fused GEMM epilogue.
enum kfamd_act { KFAMD_ACT_NONE = 0, KFAMD_ACT_RELU = 1, KFAMD_ACT_GELU_TANH = 2, KFAMD_ACT_SILU = 3 };

// C[b][m][n] = act(alpha * sum_k A[b][m][k] * B[b][n][k] + bias[n]) (+ R[b][m][n])
//   A: [batch][M][K] row-major (lda, stride_a in elements), K contiguous
//   B: [batch][N][K] row-major (ldb, stride_b), K contiguous   -> "NT" (== torch F.linear)
//   C: [batch][M][N] row-major (ldc, stride_c)
//   bias: optional [N] bf16 (nullptr = none); R: optional residual, same layout as C (ldr/stride_r)
// Dispatch: the 256x256x64 MFMA tile kernel when M%256==0, N%256==0, K%64==0 and all
// pointers/leading dims are 16-byte aligned; otherwise the bounds-checked 128x128 kernel.
int kfamd_gemm_nt_bf16(const void* A, const void* B, void* C, const void* bias, const void* R,
                       int M, int N, int K, int batch,
                       long long lda, long long ldb, long long ldc, long long ldr,
                       long long stride_a, long long stride_b, long long stride_c, long long stride_r,
                       float alpha, int act, void* stream);

// Force a specific kernel (for tests/bench): variant 0 = auto, 1 = 256x256 fast path, 2 = generic.
int kfamd_gemm_nt_bf16_variant(int variant, const void* A, const void* B, void* C, const void* bias,
                               const void* R, int M, int N, int K, int batch,
                               long long lda, long long ldb, long long ldc, long long ldr,
                               long long stride_a, long long stride_b, long long stride_c,
                               long long stride_r, float alpha, int act, void* stream);

// Layout-general GEMM on the w4 MFMA template: C[b][m][n] = act(alpha * sum_k Aop[m][k] Bop[n][k]
// + bias[n]) (+ R), with
//   la = 0: A stored [M][K] (K contiguous, lda >= K)   la = 1: A stored [K][M] (M contiguous, lda >= M)
//   lb = 0: B stored [N][K] (K contiguous, ldb >= K)   lb = 1: B stored [K][N] (N contiguous, ldb >= N)
// Aux (la = lb = 0, act = gelu/silu only): second output with the pre-activation (same layout as C).
// Transposed layouts take only alpha and R (R may alias C: C += A.B). Edge tiles are handled in the
// kernel (any M, N >= 128; N % 8; K % 8 when an operand is K-contiguous; M % 8 when la = 1). Other
// shapes return KFAMD_EINVAL and the caller falls back.
int kfamd_gemm_bf16_ex(int la, int lb, const void* A, const void* B, void* C, const void* bias, const void* R,
                       void* Aux, int M, int N, int K, int batch, long long lda, long long ldb, long long ldc,
                       long long ldr, long long stride_a, long long stride_b, long long stride_c, long long stride_r,
                       float alpha, int act, void* stream);

// Split-K for problems with too few 128x128 output tiles to fill the chip: the partial products
// of K range [z*kper, (z+1)*kper) go to W[z][b][M][N] fp32 (kper % 64 == 0, splits*kper >= K),
// then kfamd_splitk_reduce applies the epilogue into bf16 C. Same shape contract as _ex at bm=128.
int kfamd_w4_splitk_nt(const void* A, const void* B, float* W, int M, int N, int K, int batch, int splits, int kper,
                       long long lda, long long ldb, long long stride_a, long long stride_b, void* stream);
int kfamd_w4_splitk_t(int la, int lb, const void* A, const void* B, float* W, int M, int N, int K, int batch,
                      int splits, int kper, long long lda, long long ldb, long long stride_a, long long stride_b,
                      void* stream);
// Stream-K (256 tile, NT, batch 1) for grids whose last wave would leave CUs idle: `grid` persistent
// blocks (one per CU), the rem = tiles % grid leftover tiles in `splits` K-splits each; W = (splits -
// 1) * rem x 256 x 256 fp32, flags = splits * rem words owned by the calling stream with a strictly
// increasing non-zero epoch per call. Epilogues as kfamd_w4_launch_nt without the Aux output.
int kfamd_w4_streamk_nt(const void* A, const void* B, void* C, const void* bias, const void* R, void* Aux, int M,
                        int N, int K, long long lda, long long ldb, long long ldc, long long ldr, float alpha, int act,
                        float* W, unsigned* flags, unsigned epoch, int grid, int splits, void* stream);
int kfamd_splitk_reduce(const float* W, void* C, const void* bias, const void* R, void* Aux, int M, int N, int batch,
                        int splits, long long ldc, long long ldr, long long stride_c, long long stride_r, float alpha,
                        int act, void* stream);

// Softmax cross-entropy (xent_bf16.hip): forward -> per-row loss and log-sum-exp (fp32); backward ->
// dlogits = (softmax - onehot) * (*g / *count) in bf16 (device scalars: no host sync).
int kfamd_xent_fwd_bf16(const void* logits, long long ld, const long long* target, float* loss, float* lse, int rows,
                        int V, long long ignore_index, void* stream);
int kfamd_xent_bwd_bf16(const void* logits, long long ld, const long long* target, const float* lse, void* grad,
                        long long ldg, int rows, int V, long long ignore_index, const float* g, const float* count,
                        void* stream);

// K-padding pack (pad_bf16.hip): dst_i[r][0:Kp] = src_i[r][0:K], zero tail, both GEMM operands in
// one launch (rows1 = 0: one matrix). Kp % 8 == 0; dst dense and 16-B aligned.
int kfamd_pad_k_bf16(const void* src0, void* dst0, long long rows0, long long ld0, const void* src1, void* dst1,
                     long long rows1, long long ld1, int K, int Kp, void* stream);

// Fused linear-backward tail: g = dy * act'(z) (bf16; z = the forward's Aux pre-activation, or its
// output y for relu), db = column sums of g (fp32, optional). act == NONE: only db = sum over rows of
// dy (g unused). [rows][cols], cols % 8 == 0, 16-B aligned. workspace: kfamd_act_grad_workspace bytes.
long long kfamd_act_grad_workspace(int rows, int cols);
// y = act(z) elementwise (n % 8 == 0, 16-B aligned): the forward activation as its own pass
int kfamd_act_fwd_bf16(const void* z, void* y, long long n, int act, void* stream);
// multi-tensor AdamW over bf16 params / grads / moments, one launch per step (kernels/adamw_bf16.hip)
int kfamd_adamw_tensor_bytes(void);
int kfamd_adamw_chunk(void);
int kfamd_adamw_bf16(const void* table, const void* owner, long long nchunks, float lr, float b1, float b2, float eps,
                     float wd, float step_size, float inv_sqrt_bc2, void* stream);
// attention backward: dq / dk / dv [B][H][T][D] (strided) packed into the fused QKV gradient
// [B][T][3][H][D] in one pass (kernels/qkv_pack_bf16.hip)
int kfamd_qkv_pack_bf16(const void* dq, const void* dk, const void* dv, void* out, int B, int T, int H, int D,
                        long long qb, long long qh, long long qt, long long kb, long long kh, long long kt,
                        long long vb, long long vh, long long vt, void* stream);
int kfamd_act_grad_bf16(const void* dy, const void* z, void* g, float* db, float* workspace, int rows, int cols,
                        int act, void* stream);
// the same with db written as bf16 when db_bf16 (fp32 accumulation)
int kfamd_act_grad_bf16_v2(const void* dy, const void* z, void* g, void* db, int db_bf16, float* workspace, int rows,
                           int cols, int act, void* stream);
// db[c] = sum over b < nblk of ws[b][c] (fp32 partials; db fp32, or bf16 when db_bf16)
int kfamd_colsum_finalize(const float* ws, void* db, int db_bf16, int nblk, int cols, void* stream);
// A linear layer's dgrad through the previous layer's activation, one GEMM (gemm_w4.h DACT):
// G[M][N] = (dY[M][K] . W[K][N]) * act'(Z[M][N]) (dY K-contiguous with row stride lda, W row-major
// [K][N] with row stride ldb, Z / G row strides ldz / ldg), and when db is given the column sums of G
// (the previous layer's bias gradient; ws: kfamd_w4_dgrad_act_workspace bytes). M, N multiples of
// 256, K of 64, 16-B rows; KFAMD_EINVAL otherwise (callers fall back to the GEMM + act-grad pass).
// Two weight gradients in one launch: C_i[M_i][N] = A_i^T . B_i, A_i [K][M_i] (row stride lda_i), B_i
// [K][N] (ldb_i), C_i row stride ldc_i (kernels/tu/w4_wgrad_pair.hip).
int kfamd_w4_wgrad_pair(const void* A1, const void* B1, void* C1, int M1, long long lda1, long long ldb1,
                        long long ldc1, const void* A2, const void* B2, void* C2, int M2, long long lda2,
                        long long ldb2, long long ldc2, int N, int K, void* stream);
// the same with problem 2's own width N2 and, for splits > 1, K split in kper pieces with the in-kernel
// fixup (W: splits x tiles fp32 256 x 256 partials, cnt: tiles arrival counters, zero on entry and exit)
int kfamd_w4_wgrad_pair_v2(const void* A1, const void* B1, void* C1, int M1, long long lda1, long long ldb1,
                           long long ldc1, const void* A2, const void* B2, void* C2, int M2, long long lda2,
                           long long ldb2, long long ldc2, int N, int N2, int K, int splits, int kper, float* W,
                           unsigned* cnt, void* stream);
long long kfamd_w4_dgrad_act_workspace(int M, int N);
int kfamd_w4_dgrad_act(const void* dy, const void* w, void* g, const void* z, int M, int N, int K, long long lda,
                       long long ldb, long long ldg, long long ldz, int act, float* ws, void* db, int db_bf16,
                       void* stream);

// LayerNorm forward over the last dim (hidden). x,y: [rows][hidden] bf16 (row stride = hidden).
// gamma/beta: [hidden] bf16 (beta may be null). mean/rstd: optional fp32 [rows] (saved for bwd).
int kfamd_layernorm_fwd_bf16(const void* x, const void* gamma, const void* beta, void* y,
                             float* mean, float* rstd, int rows, int hidden, float eps, void* stream);

// RMSNorm forward: y = x * rsqrt(mean(x^2)+eps) * gamma. rstd optional.
int kfamd_rmsnorm_fwd_bf16(const void* x, const void* gamma, void* y, float* rstd,
                           int rows, int hidden, float eps, void* stream);

// LayerNorm backward. dx: [rows][hidden] bf16. dgamma/dbeta: fp32 [hidden] (fully written).
// workspace: fp32 scratch of kfamd_layernorm_bwd_workspace(rows, hidden) bytes.
long long kfamd_layernorm_bwd_workspace(int rows, int hidden);
int kfamd_layernorm_bwd_bf16(const void* dy, const void* x, const void* gamma, const float* mean,
                             const float* rstd, void* dx, float* dgamma, float* dbeta,
                             float* workspace, int rows, int hidden, void* stream);
// the same with dgamma / dbeta written as bf16 when dgb_bf16 (fp32 accumulation)
// v3: dres (optional, [rows][hidden] bf16, not aliasing dx): dx = dres + the LayerNorm input
// gradient (a pre-norm residual stream's two gradient contributions in one store)
int kfamd_layernorm_bwd_bf16_v3(const void* dy, const void* dres, const void* x, const void* gamma,
                                const float* mean, const float* rstd, void* dx, void* dgamma, void* dbeta,
                                int dgb_bf16, float* workspace, int rows, int hidden, void* stream);
int kfamd_layernorm_bwd_bf16_v2(const void* dy, const void* x, const void* gamma, const float* mean,
                                const float* rstd, void* dx, void* dgamma, void* dbeta, int dgb_bf16,
                                float* workspace, int rows, int hidden, void* stream);

// ---- K3: one-shot all-reduce over peer-visible buffers ------------------------------------------
enum kfamd_dtype { KFAMD_DTYPE_F32 = 0, KFAMD_DTYPE_BF16 = 1 };
// out[r] = sum over ranks of in[*] (fp32 accumulation in rank order: bit-identical on every rank).
// inputs/flags: nranks pointers (peer-visible: same device, peer-access or IPC-opened), 16-B
// aligned; outputs: rank-indexed, only [rank0, rank0 + launch_ranks) are written. One launch serves
// launch_ranks ranks (1 per device in real use; several to simulate ranks on one GPU). flags[r]:
// kfamd_allreduce_oneshot_flag_bytes(nranks, nblocks) zeroed bytes per rank, reused across calls
// with epoch = 1, 2, 3, ... (same nblocks every call). *timeout is set if a peer never arrived.
long long kfamd_allreduce_oneshot_flag_bytes(int nranks, int nblocks);
int kfamd_allreduce_oneshot_blocks(long long n, int dtype);
// Barrier deadline per call (default 5000 ms); a missed deadline sets *timeout and NaN-poisons the output.
void kfamd_allreduce_oneshot_set_timeout_ms(int ms);
int kfamd_allreduce_oneshot(const void* const* inputs, void* const* outputs, uint32_t* const* flags,
                            int nranks, int rank0, int launch_ranks, long long n, int dtype,
                            unsigned epoch, int nblocks, unsigned* timeout, void* stream);

// Two-shot (reduce-scatter + all-gather) for mid-size messages: inputs peer-visible
// and overwritten in place (rank r's slice r becomes the reduced slice), outputs per rank (need not be
// peer-visible). Same flags / epochs / timeout contract as the one-shot (flag arrays are shared).
int kfamd_allreduce_twoshot_blocks(long long n, int dtype, int nranks);
int kfamd_allreduce_twoshot(void* const* inputs, void* const* outputs, uint32_t* const* flags, int nranks, int rank0,
                            int launch_ranks, long long n, int dtype, unsigned epoch, int nblocks, unsigned* timeout,
                            void* stream);

// HIP IPC registration for one-process-per-GPU ranks (64-byte handles exchanged by the caller).
int kfamd_ipc_alloc(long long bytes, int uncached, void** ptr, void* handle64);
int kfamd_ipc_open(const void* handle64, void** ptr);
int kfamd_ipc_close(void* ptr);
int kfamd_ipc_free(void* ptr);
int kfamd_copy_async(void* dst, const void* src, long long bytes, void* stream);

// Library identity (for the loud "native code loaded" check).
const char* kfamd_build_info(void);

// Flash attention (attention_bf16.hip), bf16 I/O, fp32 softmax, head dim D = 64 or 128.
// Tensors are [B][H][T][D] views with element strides (b, h, t) (multiples of 8) and D contiguous;
// strides[3 * i + {0, 1, 2}] for tensor i in the order q, k, v, o (forward) or q, k, v, o, do, dq,
// dk, dv (backward). lse: f32 [B][H][T] (written by the forward, read by the backward).
// causal: key <= query. The backward zeroes and uses `workspace` (kfamd_attn_bwd_workspace bytes).
int kfamd_attn_fwd_bf16(const void* q, const void* k, const void* v, void* o, void* lse, int B, int H, int T,
                        int D, float scale, int causal, const long long* strides, void* stream);
long long kfamd_attn_bwd_workspace(int B, int H, int T, int D);
int kfamd_attn_bwd_bf16(const void* q, const void* k, const void* v, const void* o, const void* dout,
                        const void* lse, void* dq, void* dk, void* dv, void* workspace, int B, int H, int T,
                        int D, float scale, int causal, const long long* strides, void* stream);

#ifdef __cplusplus
}
#endif
