/*
 * medvae_hip.h -- C ABI of the MI355X (gfx950) conv-VAE training hot path.
 *
 * The reference (parsakzr/medvae-disentangled-multimodal) is pure Python/PyTorch: it has no FFI,
 * so each entry point below replaces the ATen call(s) that the named reference line issues on its
 * CPU path. The Python package medvae_disentangled_multimodal_amd binds these with ctypes (see
 * INTEGRATION.md) behind the reference's own model / LightningModule API.
 *
 * Conventions
 *   - all tensors are fp32 device pointers (HBM), activations NHWC ([n][h][w][c], c contiguous),
 *     conv weights KRSC ([cout][kh][kw][cin], i.e. torch channels_last OIHW);
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream);
 *   - kernels never allocate: scratch comes in `workspace` (size from the *_workspace_bytes query);
 *   - return 0 on success, MVAE_EINVAL (-1) / MVAE_EWORKSPACE (-2) on a bad argument, or the
 *     hipError_t of a failed launch; mvae_last_error() describes the last failure (per thread);
 *   - every reduction is two-stage and fixed-order: results are bitwise reproducible.
 */
#ifndef MEDVAE_HIP_H
#define MEDVAE_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVAE_OK 0
#define MVAE_EINVAL (-1)
#define MVAE_EWORKSPACE (-2)

const char* mvae_last_error(void);
int mvae_abi_version(void);

/* Process-wide GEMM arithmetic for all convolution / GEMM entry points below:
 * 0 = 3xBF16 fp32 emulation (default; the reference's precision=32 training),
 * 1 = bf16 operands, fp32 accumulation and fp32 outputs (the reference's precision="bf16-mixed"
 *     autocast runs these convolutions/bmm in bf16; main.py trainer precision flag). */
int mvae_set_math_mode(int mode);
int mvae_get_math_mode(void);
/* Dropout salt (device pointer to one uint64, or NULL): mixed into the seed of every following GroupNorm dropout
 * mask (ResnetBlock nn.Dropout, encoder_decoder.py:163). Lets a captured HIP graph of a training step draw fresh
 * masks per replay: the graph advances the salt on the device; the frozen per-launch seeds stay valid. */
int mvae_set_dropout_salt(const void* salt_dev);

/* ---- convolutions (implicit GEMM on MFMA, 3xBF16 split arithmetic, fp32 accumulate) ------------
 * Replaces nn.Conv2d forward in ResnetBlock/AttnBlock/Encoder/Decoder
 * (src/models/encoder_decoder.py:123-146,76-81,250-299,356-418), Downsample's F.pad + stride-2 conv
 * (:184-188, mode 0 with pad_t=pad_l=0 and zero fill beyond H/W) and Upsample's F.interpolate +
 * conv (:205-209, mode 1). mode 2 = transposed gather (input gradient of a strided conv).
 * y = conv(x) + bias[cout] + residual (residual: ResnetBlock/AttnBlock skip add, :170, :107).
 * mode | MVAE_CONV_WSPLIT: w is pre-split (mvae_split_bf16 layout; cin % 4 == 0) -- the 3xBF16 hi/lo split of
 * the weight operand is done once per step instead of in every workgroup's staging. */
#define MVAE_CONV_WSPLIT 16
/* mode | MVAE_CONV_XSPLIT (mode 0, and mvae_conv2d_wgrad_nhwc mode 0): x is pre-split the same way -- the
 * GroupNorm output written by mvae_group_norm_fwd_nhwc(y_split=1), whose only consumers are convolutions. */
#define MVAE_CONV_XSPLIT 32
/* mode | MVAE_CONV_XSPLIT with mode 2 (input gradient): dy (the gathered operand) is pre-split the same way
 * (mvae_split_bf16 of the conv's output gradient, done once for both backward GEMMs). */
/* wgrad mode | MVAE_CONV_DYSPLIT: dy (the dY^T operand) is pre-split; the fused bias gradient sums hi + lo. */
#define MVAE_CONV_DYSPLIT 64
/* mode | MVAE_CONV_BF16 (modes 0 and 2, bf16 math mode only): the gathered operand (x, or dy for mode 2) and w are
 * packed bf16 (mvae_pack_bf16 / the weight-prep entry points with split = 2; cin % 8 == 0): the GEMM stages them
 * into LDS by DMA (no staging registers or conversion) in 64-deep K-tiles -- Lightning's bf16-mixed convolution
 * (configs/config.yaml precision, main.py:86-99) with fp32 accumulation and fp32 output. */
#define MVAE_CONV_BF16 128
/* mode | MVAE_CONV_PLANAR (modes 0 and 2, default 3xBF16 math mode): the gathered operand and w are planar 3xBF16 --
 * a bf16 hi plane (hi = bf16(v)) followed by the lo plane (lo = bf16(v - hi)) of the same element count
 * (mvae_split_planar, GroupNorm y_split 3, weight prep split 3) -- staged by LDS-DMA into hi and lo images. */
#define MVAE_CONV_PLANAR 256
int mvae_conv2d_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y,
                     int nb, int h, int w_, int cin, int cout, int kh, int kw, int stride, int pad_t,
                     int pad_l, int ho, int wo, int mode, void* stream);
/* Direct 3x3 / stride-1 / pad-1 convolution at 32 input and 32 output channels (the 28x28 level of the c3 model,
 * hidden 32; encoder_decoder.py:123-146): a workgroup stages a band of input rows with its halo once into LDS and
 * runs the 9 taps as 16x16x32 MFMA products from it (no per-K-tile gather). y = conv(x, w) [+ bias][+ residual];
 * mode | MVAE_CONV_DGRAD_DIRECT: the input gradient instead -- x := dy, y := dx, w = the forward conv's weights
 * (flipped and transposed inside), no bias / residual / split weights. mode | MVAE_CONV_XSPLIT / MVAE_CONV_WSPLIT as
 * for mvae_conv2d_nhwc. NHWC fp32, KRSC weights, W <= 62. Arithmetic = the process-wide GEMM math mode. */
#define MVAE_CONV_DGRAD_DIRECT 512
int mvae_conv2d_direct32_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y,
                              int n, int h, int w_, int mode, void* stream);
/* mvae_conv2d_nhwc with a split-K workspace (same nn.Conv2d forward / input-gradient semantics): a launch whose
 * output tiles leave most of the chip idle for a partial round (small spatial sizes at wide channels, e.g. the 7x7
 * level at 512 channels of BetaVAE at 28x28) splits K over `workspace` (fp32 partials, summed in a fixed order
 * with bias / residual: deterministic). Size it with mvae_conv2d_split_workspace_bytes (0 = never splits). */
int mvae_conv2d_ws_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y,
                        int nb, int h, int w_, int cin, int cout, int kh, int kw, int stride, int pad_t,
                        int pad_l, int ho, int wo, int mode, float* workspace, size_t workspace_bytes, void* stream);
size_t mvae_conv2d_split_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo);
/* mvae_conv2d_nhwc that also emits, from the GEMM epilogue, the GroupNorm statistics of y for the
 * Normalize that consumes it (ResnetBlock conv1 -> norm2, block output -> next norm1, ...,
 * encoder_decoder.py:141-170): gn_part = [nb*ho*wo/32][cout/4][2] fp64 {sum y, sum y^2} over 32 pixels
 * x 4 channels (see mvae_group_norm_fwd_part_nhwc). Needs ho*wo % 32 == 0, cout % 4 == 0, 16-B aligned
 * y / residual / bias, cin % 4 == 0. */
int mvae_conv2d_gnstats_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y,
                             int nb, int h, int w_, int cin, int cout, int kh, int kw, int stride, int pad_t,
                             int pad_l, int ho, int wo, int mode, double* gn_part, void* stream);

/* Input gradient of a stride-1 conv (mode 2 of mvae_conv2d_nhwc, wt = [cin][kh][kw][cout]) whose input was
 * y = silu?(GroupNorm(gn_x)) (ResnetBlock norm1/norm2 -> conv1/conv2, norm_out -> conv_out;
 * encoder_decoder.py:141-163, :318-328): the GEMM epilogue also emits the GroupNorm backward partials
 * part = [nb*h*w/32][cin][2] fp64 {sum dyn, sum dyn*xhat}, dyn = dx*silu'(.), consumed by
 * mvae_group_norm_bwd_part_nhwc. Replaces the reduction half of GroupNorm's backward
 * (aten::native_group_norm_backward). No dropout in between; h*w % 32 == 0, (cin/groups) % 4 == 0.
 * w_split flags: bit 0 = wt pre-split (mvae_split_bf16 layout), bit 1 = dy pre-split. */
int mvae_conv2d_dgrad_gnbwd_nhwc(const float* dy, const float* wt, float* dx, int nb, int ho, int wo, int cout,
                                 int cin, int kh, int kw, int pad_t, int pad_l, int h, int w_, int w_split,
                                 const float* gn_x, const float* mean, const float* rstd, const float* gamma,
                                 const float* beta, int groups, int silu, double* part, void* stream);

/* Weight gradient of mvae_conv2d_nhwc (modes 0/1): dw = beta*dw + sum_pixels dy (x) x, and (if dbias
 * is non-null) the bias gradient dbias = beta*dbias + sum_pixels dy, computed from the same staged dy.
 * Replaces the weight/bias half of aten::convolution_backward for the convolutions above. */
int mvae_conv2d_wgrad_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb, int h, int w_,
                           int cin, int cout, int kh, int kw, int stride, int pad_t, int pad_l, int ho,
                           int wo, int mode, float* workspace, size_t workspace_bytes, void* stream);
size_t mvae_conv2d_wgrad_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo);

/* Weight (+ bias) gradient of a 3x3 / stride-1 / pad-1 conv with 1 <= cout <= 4 (Decoder.conv_out,
 * src/models/encoder_decoder.py:418-419): each x element read once and scattered into its 9 taps
 * (a cout-row implicit GEMM would stream the 9x im2col for 3 useful rows). Same contract as
 * mvae_conv2d_wgrad_nhwc (dw = beta*dw + ..., dbias optional); x_split = 1: x holds split4_bf16 groups
 * (x = hi + lo). cin % 4 == 0, x 16-B aligned. Deterministic (fixed-order partials). */
int mvae_conv2d_wgrad_small_cout_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb,
                                      int h, int w_, int cin, int cout, int x_split, void* workspace,
                                      size_t workspace_bytes, void* stream);
size_t mvae_conv2d_wgrad_small_cout_workspace_bytes(int nb, int cin);
/* Weight (+ bias) gradient of a 3x3 / stride-1 / pad-1 conv with cin, cout in {32, 64} (the 28x28 / 14x14 levels
 * of the c3 disentangled model): replaces the implicit-GEMM form of convolution_backward's weight half there.
 * Per-tap 32x32x16 MFMA products over LDS-resident row bands, persistent grid, fixed-order partial reduction.
 * dw, dbias (optional) accumulate with beta. x_split: x holds split4_bf16 groups. Math modes 0 (3xBF16) and 1
 * (bf16); the exact-fp32 mode is rejected (use mvae_conv2d_wgrad_nhwc). */
int mvae_conv2d_wgrad_direct_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb, int h,
                                  int w, int cin, int cout, int x_split, void* workspace, size_t workspace_bytes,
                                  void* stream);
size_t mvae_conv2d_wgrad_direct_workspace_bytes(int nb, int h, int w, int cin, int cout);

/* Input gradient of a stride-2 conv (Downsample, encoder_decoder.py:184-188) by dx parity class: each
 * class is a dense stride-1 conv of dy [nb][ho][wo][cout] with its own <= 2x2 taps of wt [cin][kh][kw][cout]
 * (mvae_conv_weight_transpose), written interleaved into dx [nb][h][w_][cin] (h, w_ even): the useful
 * MACs only, vs mode 2's transposed gather where 3/4 of the taps hit stride holes.
 * workspace >= 4*kh*kw*cin*cout bytes (per-class weights). w_split flags: bit 0 = wt pre-split, bit 1 = dy
 * pre-split (mvae_split_bf16 layout; cout % 4 == 0); w_split = 4: dy and wt packed bf16 (MVAE_CONV_BF16). */
int mvae_conv2d_dgrad_stride2_nhwc(const float* dy, const float* wt, float* dx, int nb, int h, int w_, int cin,
                                   int cout, int kh, int kw, int pad_t, int pad_l, int ho, int wo, int w_split,
                                   float* workspace, size_t workspace_bytes, void* stream);

/* Upsample's conv (nearest x2 then 3x3, stride 1, pad 1; encoder_decoder.py:194-209) in sub-pixel form:
 * output parity class (ph, pw) is a 2x2 conv of the low-resolution x [nb][h][w_][cin] with the tap-summed
 * weights w4 [4][cout][2][2][cin] (mvae_conv_weight_upsample_fwd), written interleaved into
 * y [nb][2h][2w_][cout] -- 4/9 of the reference's MACs, no upsampled intermediate. Same result as
 * mvae_conv2d_nhwc mode 1 up to fp32 summation order. w_split = 1: w4 pre-split; 2: x and w4 packed bf16
 * (MVAE_CONV_BF16). */
int mvae_conv2d_upsample_nhwc(const float* x, const float* w4, const float* bias, const float* residual, float* y,
                              int nb, int h, int w_, int cin, int cout, int w_split, void* stream);
int mvae_conv_weight_upsample_fwd(const float* w, float* w4, int cout, int cin, int split, void* stream);
/* Its weight (+ bias) gradient: per-class [cout] x [4*cin] GEMMs over the class pixels, deterministic
 * split-K partials in the workspace, then a fixed-order combine into dw [cout][3][3][cin] (beta-accumulate). */
int mvae_conv2d_wgrad_upsample_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb,
                                    int h, int w_, int cin, int cout, float* workspace, size_t workspace_bytes,
                                    void* stream);
size_t mvae_conv2d_wgrad_upsample_workspace_bytes(int nb, int h, int w_, int cin, int cout);

/* Winograd F(m x m, 3x3) form of a 3x3 / stride-1 / pad-1 conv, m = `tile` in {2, 4} (ResnetBlock conv1 / conv2 and
 * the mid blocks at the 8x8 / 16x16 levels, encoder_decoder.py:123-170; forward, input gradient, weight gradient),
 * every math mode (mvae_set_math_mode); a = m + 2, P = a^2 transformed positions, T = nb (h/m) (w/m) output tiles. Stages on the
 * stream: U = G g G^T of the filters, V = B^T d B of the input's a x a patches, M_xi = V_xi U_xi^T for the P positions
 * (one batched MFMA GEMM: P / (9 m^2) of the direct conv's MACs -- 4/9 at m = 2, 1/4 at m = 4), output A^T M A
 * (+ bias, + residual, + the following GroupNorm's statistics). The input gradient is the same conv of dy with the
 * flipped, transposed filters (weight_transform dgrad = 1) and may emit the GroupNorm backward partials of
 * mvae_conv2d_dgrad_gnbwd_nhwc (output_gnbwd). V, U, D': 16 B per 4 values in the math mode's pre-split layout --
 * split4_bf16 in the 3xBF16 and bf16 modes (the bf16 GEMM reads the hi halves), the split4 bit split (upper / lower 16
 * bits of each fp32 word) in the exact fp32 mode, where x_split / dy_split must be 0; M: fp32. Conditions: channel counts
 * % 4 == 0, 16-B aligned operands, each transformed operand < 4 GiB; the statistics / GroupNorm-backward forms need
 * h % 4 == 0 and w in {8, 16} or a multiple of 32.
 *   weight_transform: w [cout][3][3][cin] -> u [P][cout][cin] (dgrad 0) or [P][cin][cout] (dgrad 1)
 *   input_transform:  x [nb][h][w][c] (fp32, or split4_bf16 groups when x_split) -> v [P][T][c]
 *   gemm:             m [P][tiles][n_out] = v . u^T over k_in
 *   output_transform: m -> y [nb][h][w][n] (+ bias[n]) (+ residual [nb][h][w][n]); gn_part as mvae_conv2d_gnstats_nhwc
 *   output_gnbwd:     m -> dx, part as mvae_conv2d_dgrad_gnbwd_nhwc (x, mean, rstd, gamma, beta: that GroupNorm's)
 * Weight gradient, F(3x3, m x m) on the same tiles: dw = beta*dw + G^T M G with M_xi = sum_tiles D'_xi (x) V_xi,
 * D' = A D A^T of the m x m output-gradient tiles, V the forward's input transform:
 *   dy_transform:  dy [nb][h][w][k] (fp32, or split4_bf16 groups when dy_split) -> d [P][T][k] split4_bf16
 *   wgrad_gemm:    m [P][cout][cin] = sum over tiles d^T v (split over the tiles within workspace:
 *                  mvae_gemm_workspace_bytes(cout, cin, tiles, P))
 *   wgrad_output:  dw [cout][3][3][cin] = beta*dw + G^T m G
 * The conv bias gradient is not produced here (mvae_bias_grad, or the GroupNorm backward that split dy). */
int mvae_winograd_weight_transform(const float* w, void* u, int cin, int cout, int dgrad, int tile, void* stream);
int mvae_winograd_input_transform(const float* x, void* v, int nb, int h, int w, int c, int x_split, int tile,
                                  void* stream);
/* input_transform of silu?(GroupNorm(x)) with the normalization applied on load (x = the GroupNorm's INPUT, scale /
 * shift [nb][c] = rstd * gamma, beta - mean * rstd * gamma from mvae_group_norm_stats_nhwc): the GroupNorm output that
 * only feeds this conv is never written (the SURVEY §7 GroupNorm+SiLU-into-the-conv-operand fusion, on the Winograd
 * form's one read of its input). */
int mvae_winograd_input_transform_gn(const float* x, const float* scale, const float* shift, int silu, void* v, int nb,
                                     int h, int w, int c, int tile, void* stream);
int mvae_winograd_gemm(const void* v, const void* u, float* m, long long tiles, int k_in, int n_out, int tile,
                       void* stream);
int mvae_winograd_output_transform(const float* m, const float* bias, const float* residual, float* y, double* gn_part,
                                   int nb, int h, int w, int n, int tile, void* stream);
int mvae_winograd_output_gnbwd(const float* m, float* dx, const float* x, const float* mean, const float* rstd,
                               const float* gamma, const float* beta, int groups, int silu, double* part, int nb, int h,
                               int w, int n, int tile, void* stream);
int mvae_winograd_dy_transform(const float* dy, void* d, int nb, int h, int w, int k, int dy_split, int tile,
                               void* stream);
// Both backward transforms of dy in one pass (a conv whose input and weight gradients both run the Winograd form):
// v = mvae_winograd_input_transform(dy) and d = mvae_winograd_dy_transform(dy), each [a^2][T][k] split4_bf16.
// Replaces the two separate passes over dy of the conv backward (encoder_decoder.py ResnetBlock convs, autograd).
int mvae_winograd_dy_transforms(const float* dy, void* v, void* d, int nb, int h, int w, int k, int dy_split, int tile,
                                void* stream);
int mvae_winograd_wgrad_gemm(const void* d, const void* v, float* m, long long tiles, int cout, int cin, int tile,
                             float* workspace, size_t workspace_bytes, void* stream);
int mvae_winograd_wgrad_output(const float* m, float* dw, float beta, int cout, int cin, int tile, void* stream);
/* The Upsample conv (nearest x2, then 3x3 / pad 1: encoder_decoder.py:194-209, Upsample) on the Winograd form: four 3x3 /
 * pad-1 class convs on the low-resolution input x [nb][h][w][cin], one per output parity class (p, q) -- class kernel
 * K_pq = the sub-pixel form's tap sums embedded in a 3x3 support -- sharing x's input transform:
 *   upsample_weights: w [cout][3][3][cin] -> kc [4 cout][3][3][cin] (row pq * cout + k); weight_transform(kc, 4 cout)
 *                     then gives U (forward, dgrad 0) or U' (input gradient, dgrad 1)
 *   gemm(V of x, U, n_out = 4 cout) -> output_transform_upsample -> y [nb][2h][2w][cout] (+ bias)
 *   dy_transforms_upsample: dy [nb][2h][2w][cout] -> V' (nullable) and D', each [a^2][T][4 cout] from the four class
 *                     sub-images dy[2i + p][2j + q]; gemm(V', U', k_in = 4 cout, n_out = cin) -> output_transform -> dx
 *   wgrad_gemm(D', V of x, cout = 4 cout) -> wgrad_output -> dkc [4 cout][3][3][cin]; upsample_fold: dw = beta * dw +
 *                     each class kernel's gradient summed onto the taps it was built from */
int mvae_winograd_upsample_weights(const float* w, float* kc, int cin, int cout, void* stream);
int mvae_winograd_upsample_fold(const float* dkc, float* dw, float beta, int cin, int cout, void* stream);
int mvae_winograd_output_transform_upsample(const float* m, const float* bias, float* y, int nb, int h, int w, int cout,
                                            int tile, void* stream);
int mvae_winograd_dy_transforms_upsample(const float* dy, void* v, void* d, int nb, int h, int w, int cout, int tile,
                                         void* stream);

/* 3xBF16 operand pre-split (same bytes as the fp32 tensor): per 4 values hi0..hi3 lo0..lo3 bf16,
 * hi = bf16(x) (round to nearest even), lo = bf16(x - hi). The weight-prep entry points below take
 * `split` to emit this layout directly (along their contiguous dimension, which must be % 4). */
int mvae_split_bf16(const float* x, void* y, long long n, void* stream);
/* Packed bf16 (round to nearest even) of n fp32 values (n % 8 == 0, 16-B aligned): the bf16-mixed mode's GEMM
 * operands (MVAE_CONV_BF16). The weight-prep entry points take split = 2 to emit it directly. */
int mvae_pack_bf16(const float* x, void* y, long long n, void* stream);
/* Packed bf16 of a conv output gradient dy [rows][n] (n % 4 == 0) and, from the same pass, its bias gradient
 * out[n] = beta*out[n] + sum_rows dy (fp64 partials, fixed order; workspace mvae_bias_grad_workspace_bytes). */
int mvae_pack_bf16_colsum(const float* x, void* y, long long rows, int n, float* out, float beta, void* workspace,
                          size_t workspace_bytes, void* stream);
/* Planar 3xBF16 (MVAE_CONV_PLANAR) of n fp32 values (n % 4 == 0): y = [hi plane: n bf16][lo plane: n bf16]. */
int mvae_split_planar(const float* x, void* y, long long n, void* stream);
/* mvae_pack_bf16_colsum writing dy planar 3xBF16 instead of packed bf16. */
int mvae_split_planar_colsum(const float* x, void* y, long long rows, int n, float* out, float beta, void* workspace,
                             size_t workspace_bytes, void* stream);

/* Weight re-layouts for the input gradient: KRSC -> [cin][kh][kw][cout]; and the 4x4 tap-summed
 * kernel [cin][4][4][cout] for Upsample's conv (encoder_decoder.py:205-209). */
int mvae_conv_weight_transpose(const float* w, float* wt, int cout, int kh, int kw, int cin, int split, void* stream);
/* All of a step's dgrad weight re-layouts in one launch: `table` (device memory) holds n descriptors sorted by
 * block0, each one mvae_conv_weight_transpose (w [cout][rs][cin] -> wt [cin][rs][cout] in format `split`) over
 * ceil(cin/64) * ceil(cout/64) * rs workgroups starting at block0; total_blocks = the sum. */
typedef struct {
  const float* w;
  float* wt;
  int cout, rs, cin, split;
  int block0, pad0;
} mvae_wt_desc;
int mvae_conv_weight_transpose_batched(const mvae_wt_desc* table, int n, int total_blocks, void* stream);
int mvae_conv_weight_upsample_dgrad(const float* w, float* wt, int cout, int cin, int split, void* stream);

/* Bias gradient: out[n] = beta*out[n] + sum_rows x[row*ld + n] (conv bias, encoder_decoder.py:123-146). */
int mvae_bias_grad(const float* x, long long rows, int n, long long ld, float* out, float beta,
                   void* workspace, size_t workspace_bytes, void* stream);
size_t mvae_bias_grad_workspace_bytes(long long rows, int n);

/* ---- batched GEMM (AttnBlock's torch.bmm pair, encoder_decoder.py:90-103) ----------------------
 * C[b] = alpha*op(A[b]) op(B[b]) + bias + residual[b] + beta*C[b], row-major.
 * trans_a: A stored [K][M]; trans_b: B stored [N][K]. */
int mvae_gemm_strided_batched(int trans_a, int trans_b, int m, int n, int k, float alpha,
                              const float* A, long long lda, long long stride_a, const float* B,
                              long long ldb, long long stride_b, float beta, float* C, long long ldc,
                              long long stride_c, int batch, const float* bias, const float* residual,
                              long long ldr, long long stride_r, float* workspace,
                              size_t workspace_bytes, void* stream);
size_t mvae_gemm_workspace_bytes(int m, int n, int k, int batch);

/* Row softmax of the attention scores (F.softmax(w_, dim=2), encoder_decoder.py:97) and its grad. */
int mvae_softmax_rows(const float* x, float* y, long long rows, int n, void* stream);
int mvae_softmax_rows_bwd(const float* y, const float* dy, float* dx, long long rows, int n, void* stream);

/* Fused single-tile attention core for n <= 64 tokens per image (the 7x7 / 8x8 mid AttnBlocks,
 * encoder_decoder.py:83-107): o = softmax(q k^T * scale, dim=2) v in ONE launch per direction, one workgroup per
 * image, the n x n scores kept in LDS. q, k, v, o: [batch][n][c] fp32 (channels contiguous), c % 64 == 0;
 * lse: [batch][64] fp32, the row log-sum-exp of the scaled scores written by the forward and read by the backward
 * (which recomputes the scores: no score tensor in HBM). Products in the process-wide GEMM arithmetic. */
int mvae_attention_small_fwd(const float* q, const float* k, const float* v, float* o, float* lse, int batch, int n,
                             int c, float scale, void* stream);
int mvae_attention_small_bwd(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                             float* dq, float* dk, float* dv, int batch, int n, int c, float scale, void* stream);

/* Query-block fused attention for 64 <= n <= 256 tokens, n % 64 == 0, c % 128 == 0 (c4 / c5's 16x16 AttnBlocks and the
 * 8x8 mid blocks at C = 2048, encoder_decoder.py:83-107): one workgroup per (64-query block, image).
 * fwd: o = softmax(q k^T * scale, dim=2) v in one launch; p [batch][n][n] receives P (the backward's saved tensor).
 * bwd: from P and dout: dq = dS k and ds [batch][n][n] = scale * P o (dP - rowsum(P o dP)), dP = dout v^T, in one
 * launch; dv = P^T dout and dk = ds^T q are left to mvae_gemm_strided_batched (sums over every query block). */
int mvae_attention_tile_fwd(const float* q, const float* k, const float* v, float* o, float* p, int batch, int n, int c,
                            float scale, void* stream);
int mvae_attention_tile_bwd(const float* k, const float* v, const float* dout, const float* p, float* dq, float* ds,
                            int batch, int n, int c, float scale, void* stream);

/* ---- GroupNorm (+SiLU, +inverted dropout) -------------------------------------------------------
 * Normalize() = nn.GroupNorm(min(32,C), C, eps=1e-6) (encoder_decoder.py:28-33) fused with
 * nonlinearity() (:13-15) and ResnetBlock's nn.Dropout (:163). mean/rstd: [nb*groups].
 * Backward ACCUMULATES into dgamma/dbeta (flat grad buffer); dx_add (nullable, [nb][hw][c]) is the
 * gradient of x from the block's other branch (ResnetBlock / AttnBlock residual, encoder_decoder.py:
 * 107,170), summed into dx in the same pass (replaces autograd's separate gradient add).
 * y_split = 1: y is written in the pre-split 3xBF16 operand layout (mvae_split_bf16) for a following
 * convolution (MVAE_CONV_XSPLIT); 2: packed bf16 (MVAE_CONV_BF16); 3: planar 3xBF16 (MVAE_CONV_PLANAR) -- the
 * backward never reads y. */
int mvae_group_norm_fwd_nhwc(const float* x, const float* gamma, const float* beta, float* y, float* mean,
                             float* rstd, int nb, int hw, int c, int groups, float eps, int silu,
                             float drop_p, unsigned long long seed, int y_split, void* workspace,
                             size_t workspace_bytes, void* stream);
int mvae_group_norm_bwd_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                             const float* mean, const float* rstd, float* dx, const float* dx_add,
                             float* dgamma, float* dbeta,
                             int nb, int hw, int c, int groups, int silu, float drop_p,
                             unsigned long long seed, void* workspace, size_t workspace_bytes,
                             void* stream);
size_t mvae_group_norm_workspace_bytes(int nb, int hw, int c);
/* mvae_group_norm_bwd_nhwc that also writes dx as packed bf16 (dx_packed: 2 B per element at the element offsets,
 * 8-B aligned -- the bf16-mixed GEMMs' operand format) and, when dbias is non-null, dbias[c] = bias_beta * dbias[c]
 * + sum over rows of dx (fp64 partials in cs_workspace, fixed order): the output gradient and bias gradient of the
 * convolution whose output this GroupNorm normalizes (ResnetBlock conv1 -> norm2, the next block's norm1), in the
 * same pass as dx -- replaces mvae_pack_bf16_colsum over dx (the conv bias half of convolution_backward,
 * encoder_decoder.py:141-163). x, dy, dx, dx_add 16-B aligned. dx may be null (this form, the split form and the
 * partials form): the fp32 dx is not written when the producing conv -- its only consumer -- reads the copy alone. */
int mvae_group_norm_bwd_pack_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                                  const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                                  float* dbeta, int nb, int hw, int c, int groups, int silu, float drop_p,
                                  unsigned long long seed, void* workspace, size_t workspace_bytes, void* dx_packed,
                                  float* dbias, float bias_beta, void* cs_workspace, size_t cs_workspace_bytes,
                                  void* stream);
size_t mvae_group_norm_colsum_workspace_bytes(int nb, int hw, int c);
/* The same with dx also written as split4_bf16 groups (dx_split: 4 B per element at dx's element offsets, 16-B
 * aligned; mvae_split_bf16's layout) -- the fp32-class (3xBF16) GEMMs' pre-split dY operand of the producing conv's
 * input and weight gradients (MVAE_CONV_XSPLIT / MVAE_CONV_DYSPLIT), with the conv bias gradient as above. */
/* ... with dx in fp32 only, plus the producing conv's bias gradient (the column sums of dx, accumulated with bias_beta):
 * the exact-fp32 arithmetic's and the Winograd Upsample conv's replacement for a separate column-sum pass over dy. */
int mvae_group_norm_bwd_colsum_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                                    const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                                    float* dbeta, int nb, int hw, int c, int groups, int silu, float drop_p,
                                    unsigned long long seed, void* workspace, size_t workspace_bytes, float* dbias,
                                    float bias_beta, void* cs_workspace, size_t cs_workspace_bytes, void* stream);
int mvae_group_norm_bwd_split_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                                   const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                                   float* dbeta, int nb, int hw, int c, int groups, int silu, float drop_p,
                                   unsigned long long seed, void* workspace, size_t workspace_bytes, void* dx_split,
                                   float* dbias, float bias_beta, void* cs_workspace, size_t cs_workspace_bytes,
                                   void* stream);
/* Path of mvae_group_norm_fwd_nhwc / _bwd_nhwc (process-wide): 0 = auto (small per-sample tensors -- the
 * 28x28 / 14x14 / 7x7 levels -- run the register-resident one-pass kernels: x read once per pass),
 * 1 = streaming only (statistics pass + apply pass). Both are deterministic; they agree to fp32 rounding. */
int mvae_set_group_norm_path(int mode);
/* GroupNorm statistics only, for a consumer that normalizes on load (mvae_winograd_input_transform_gn): mean / rstd
 * [nb * groups] and the apply's affine scale = rstd * gamma, shift = beta - mean * scale ([nb][c]); part (nullable):
 * the producing conv's epilogue statistics (no pass over x). mvae_group_norm_apply_nhwc materializes y = silu?(x * scale
 * + shift) from them when a deferred output must exist after all (y_split as mvae_group_norm_fwd_nhwc, no dropout). */
int mvae_group_norm_stats_nhwc(const float* x, const double* part, const float* gamma, const float* beta, float* mean,
                               float* rstd, float* scale, float* shift, int nb, int hw, int c, int groups, float eps,
                               void* workspace, size_t workspace_bytes, void* stream);
int mvae_group_norm_apply_nhwc(const float* x, const float* scale, const float* shift, float* y, int nb, int hw, int c,
                               int silu, int y_split, void* stream);
/* mvae_group_norm_bwd_nhwc (drop_p = 0) from the partials of mvae_conv2d_dgrad_gnbwd_nhwc: no reduction
 * pass over x and dy. hw % 32 == 0. */
int mvae_group_norm_bwd_part_nhwc(const float* x, const float* dy, const double* part, const float* gamma,
                                  const float* beta, const float* mean, const float* rstd, float* dx,
                                  const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c, int groups,
                                  int silu, void* workspace, size_t workspace_bytes, void* stream);
/* ... with dx also written split4_bf16 and the producing conv's bias gradient (mvae_group_norm_bwd_split_nhwc's
 * outputs; the partials from the Winograd input-gradient output transform, mvae_winograd_output_gnbwd). dx_split may be
 * null when dbias is given: the bias column sums only (mvae_group_norm_bwd_colsum_nhwc's outputs, exact fp32). */
int mvae_group_norm_bwd_part_split_nhwc(const float* x, const float* dy, const double* part, const float* gamma,
                                        const float* beta, const float* mean, const float* rstd, float* dx,
                                        const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c,
                                        int groups, int silu, void* workspace, size_t workspace_bytes, void* dx_split,
                                        float* dbias, float bias_beta, void* cs_workspace, size_t cs_workspace_bytes,
                                        void* stream);
/* 1 when the GroupNorm backward of this geometry (with_dxp: its split / packed-output forms) runs the two-pass
 * streaming chain, whose partial pass the consuming conv can supply; 0 for the one-pass resident / unit kernels. */
int mvae_group_norm_bwd_streaming(int nb, int hw, int c, int groups, int with_dxp);
/* mvae_group_norm_fwd_nhwc from the statistics the producing convolution emitted
 * (mvae_conv2d_gnstats_nhwc, part = [nb*hw/32][c/4][2] fp64): skips the statistics pass over x.
 * hw % 32 == 0, (c / groups) % 4 == 0. */
int mvae_group_norm_fwd_part_nhwc(const float* x, const double* part, const float* gamma, const float* beta, float* y,
                                  float* mean, float* rstd, int nb, int hw, int c, int groups, float eps, int silu,
                                  float drop_p, unsigned long long seed, int y_split, void* workspace,
                                  size_t workspace_bytes, void* stream);

/* ---- reparameterization / KL / reconstruction ---------------------------------------------------
 * BaseVAE.reparameterize (src/models/base_vae.py:83-87) with explicit eps; mu/logvar are channel
 * slices of the encoder output (row stride ld >= zc), torch.chunk (:76) costs nothing. */
int mvae_reparam_fwd(const float* mu, const float* logvar, long long ld, const float* eps, float* z,
                     long long npix, int zc, void* stream);
int mvae_reparam_bwd(const float* dz, const float* eps, const float* logvar, long long ld, float* dlogvar,
                     long long npix, int zc, void* stream);
/* out[0] = scale * sum(term): kind 0 = KL(N(mu,e^{lv/2})||N(0,1)) (vae_losses.py:58),
 * 1 = squared error (mse, :41), 2 = absolute error (l1, :43), 3 = -0.5*(1+lv-mu^2-e^lv)
 * (DisentangledVAELoss, disentangled_conditional_vae.py:524), adversarial terms on logits a
 * (vae_losses.py:297-352): 4 = relu(1-a), 5 = relu(1+a), 6 = a. Device scalar out, no host sync. */
int mvae_loss_reduce(int kind, const float* a, const float* b, long long ld, long long npix, int zc,
                     double scale, float* out, void* workspace, size_t workspace_bytes, void* stream);
size_t mvae_reduce_workspace_bytes(void);
int mvae_kl_bwd(const float* mu, const float* logvar, long long ld, const float* gscale, double mult,
                float* dmu, float* dlogvar, long long npix, int zc, void* stream);
int mvae_recon_bwd(int kind, const float* a, const float* b, const float* gscale, double mult, float* da,
                   long long n, void* stream);
/* DisentangledConditionalVAE.forward's latent side in one pass (src/models/disentangled_conditional_vae.py:
 * 388-398 after encode's NaN scrub, :255-301; reparameterize base_vae.py:83-87): mu = clamp(nan0(h_mu), -10, 10),
 * logvar likewise, s = exp(logvar/2), z = mu + eps*s, std = clamp(s, 1e-6, 10); outputs dense [npix][zc].
 * The backward writes the gradients of h_mu / h_logvar at row stride ld_out (the encoder output's gradient);
 * null incoming gradients count as zero. */
int mvae_latent_prep_fwd(const float* h_mu, const float* h_logvar, long long ld, const float* eps, float* mu,
                         float* logvar, float* std_out, float* z, long long npix, int zc, void* stream);
int mvae_latent_prep_bwd(const float* h_mu, const float* h_logvar, long long ld, const float* eps, const float* g_mu,
                         const float* g_logvar, const float* g_std, const float* g_z, float* d_mu, float* d_logvar,
                         long long ld_out, long long npix, int zc, void* stream);
/* DisentangledVAELoss's total (src/models/disentangled_conditional_vae.py:528-570): nt <= 4 device scalars v_i,
 * o_i = v_i if finite else 0, total = sum w_i o_i (fp32, in order) or nonfinite_total when not finite;
 * flags[0..nt] record finiteness for the backward: g_terms[i] = [v_i finite](g_i + w_i [total finite] g_total). */
int mvae_loss_combine4_fwd(const float* v0, const float* v1, const float* v2, const float* v3, float w0, float w1,
                           float w2, float w3, int nt, float nonfinite_total, float* total, float* o0, float* o1,
                           float* o2, float* o3, float* flags, void* stream);
int mvae_loss_combine4_bwd(const float* flags, float w0, float w1, float w2, float w3, int nt, const float* g_total,
                           const float* g0, const float* g1, const float* g2, const float* g3, float* g_terms,
                           void* stream);

/* ---- optimizer step over one flat buffer ----------------------------------------------------------
 * on_before_optimizer_step (lightning_module.py:468-477) + configure_gradient_clipping (:452-466) +
 * Adam/AdamW (configure_optimizers, :390-408). scalars[0] = total grad norm, scalars[1] = coef. */
int mvae_multi_tensor_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                           const int* chunk_tensor, const long long* chunk_start, const int* chunk_len,
                           int nchunks, const int* tensor_chunk_begin, int ntensors, const int* used,
                           int* step, float grad_scale, float max_norm, int do_clip, float lr, float beta1,
                           float beta2, float eps, float weight_decay, int decoupled, void* workspace,
                           size_t workspace_bytes, float* scalars, void* stream);
size_t mvae_multi_tensor_adam_workspace_bytes(int nchunks, int ntensors);

/* ---- perceptual loss (LPIPSLoss, src/losses/vae_losses.py:67-94; lpips 0.1.4 net="alex"/"vgg") ----
 * y = (a*x + b - shift[c]) * inv_scale[c]: `inputs*2-1` (a=2, b=-1) then lpips' ScalingLayer. */
int mvae_lpips_scale(const float* x, float* y, long long n, int c, float a, float b, const float* shift,
                     const float* inv_scale, void* stream);
int mvae_lpips_scale_bwd(const float* dy, float* dx, long long n, int c, float a, const float* inv_scale,
                         void* stream);
/* ReLU of the AlexNet feature slices (torchvision alexnet.features) and its gradient (from the output). */
int mvae_relu_fwd(const float* x, float* y, long long n, void* stream);
int mvae_relu_bwd(const float* y, const float* dy, float* dx, long long n, void* stream);
/* MaxPool2d(k, stride) over NHWC (AlexNet 3/2, VGG16 2/2); argmax = window index per output element
 * (first max wins, as in torch). */
int mvae_maxpool_fwd(const float* x, float* y, unsigned char* argmax, int nb, int h, int w, int c, int k, int stride,
                     void* stream);
int mvae_maxpool_bwd(const float* dy, const unsigned char* argmax, float* dx, int nb, int h, int w, int c, int k,
                     int stride, void* stream);
/* One LPIPS layer: score[b] = beta*score[b] + mean_p sum_c w[c] (f0/(|f0|+1e-10) - f1/(|f1|+1e-10))^2
 * (normalize_tensor + NetLinLayer 1x1 conv + spatial_average); c <= 512. Gradient w.r.t. f0 and (if
 * df1 != NULL) f1, scaled by gscore[b]. */
int mvae_lpips_dist(const float* f0, const float* f1, const float* w, float* score, int nb, int npix, int c,
                    float beta, void* stream);
int mvae_lpips_dist_bwd(const float* f0, const float* f1, const float* w, const float* gscore, float* df0, float* df1,
                        int nb, int npix, int c, void* stream);

/* ---- validation metrics (validation_step, src/lightning_module.py:220-300; src/utils/metrics.py:14-73) ----
 * SSIM exactly as torchmetrics 1.7.4 structural_similarity_index_measure (11x11 Gaussian, sigma 1.5,
 * k1 0.01, k2 0.03, border-cropped map): per_image[b] = mean SSIM of image b (NHWC, h, w >= 11). */
int mvae_ssim(const float* x, const float* y, int nb, int h, int w, int c, float data_range, float* per_image,
              void* stream);
/* compute_kl_metrics on [pixels][zc] latents (row stride ld): out = {kl_total, kl_mean, kl_std (unbiased),
 * kl_per_dim_mean}, where the per-"sample" sums run over the channel dim (dim 1 of the NCHW latent). */
int mvae_kl_stats(const float* mu, const float* logvar, long long ld, long long npix, int zc, float* out,
                  void* workspace, size_t workspace_bytes, void* stream);
size_t mvae_kl_stats_workspace_bytes(long long npix);

/* ---- on-device MedMNIST batches (row (f)1: MedMNISTDataset.__getitem__ + transforms + collate,
 * src/data/medmnist_data.py:16-72,186-251,319-375) ---------------------------------------------------
 * store: resident uint8 images (sample s at byte sample_offset[s], [h][w][sample_channels[s]]);
 * converts to sample_target_channels[s] (1/3), optional per-sample augmentation `aug` (12 floats per
 * sample: flip, inverse-rotation rows scaled by (w/2, h/2), brightness f / 1-f, contrast f / 1-f,
 * order, 2 pad; NULL = evaluation transform), Normalize(0.5, 0.5), zero-pads to cout channels.
 * Writes x NHWC [nb][h][w][cout], onehot [nb][n_modalities], modality_idx [nb], labels [nb]. */
int mvae_decode_batch(const unsigned char* store, const long long* sample_offset, const int* sample_channels,
                      const int* sample_target_channels, const int* sample_modality, const long long* sample_label,
                      const long long* index, const float* aug, int nb, int h, int w, int cout, int n_modalities,
                      float* x, float* onehot, long long* modality_idx, long long* labels, void* workspace,
                      size_t workspace_bytes, void* stream);
size_t mvae_decode_batch_workspace_bytes(int nb, int h);

/* Gradient of the adversarial terms (kinds 4-6) w.r.t. the logits, times gscale[0] * mult. */
int mvae_adv_bwd(int kind, const float* a, const float* gscale, double mult, float* da, long long n, void* stream);

/* ---- adversarial branch (row (f)2): NLayerDiscriminator (src/models/discriminator.py:11-82) -------
 * BatchNorm2d over NHWC rows (N*H*W) fused with LeakyReLU(slope; slope < 0 = none). training: batch
 * statistics -> mean/rstd (saved for backward), running stats updated (momentum, unbiased var) when
 * run_mean != NULL; training == 0: running statistics. Backward (training mode) accumulates into
 * dgamma/dbeta. */
int mvae_batch_norm_fwd_nhwc(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd,
                             float* run_mean, float* run_var, long long rows, int c, float eps, float momentum,
                             int training, float slope, void* workspace, size_t workspace_bytes, void* stream);
int mvae_batch_norm_bwd_nhwc(const float* x, const float* y, const float* dy, const float* gamma, const float* mean,
                             const float* rstd, float* dx, float* dgamma, float* dbeta, long long rows, int c,
                             float slope, void* workspace, size_t workspace_bytes, void* stream);
size_t mvae_batch_norm_workspace_bytes(long long rows, int c);
int mvae_leaky_relu_fwd(const float* x, float* y, float slope, long long n, void* stream);
int mvae_leaky_relu_bwd(const float* y, const float* dy, float* dx, float slope, long long n, void* stream);

/* ---- disentangled modality routing (DisentangledConditionalVAE) ------------------------------------------
 * Replaces the reference's per-sample Python loops (src/models/disentangled_conditional_vae.py:137-169 encode,
 * :255-301 decode): ONE launch per batch; each sample reads its modality id idx[b] (int64, device; ids >= nm
 * use modality nm-1 like :142-146 / :260-265) and runs only that modality's layers. c (max channels) must be 3
 * (the reference's channel map {0:1, 1:3, 2:3, 3:1, 4:3}); nm <= 8; the image must fit the LDS tiles
 * ((4*(h+2)*(w+2) + h*w) * c * 4 bytes <= 160 KiB). Parameter tables are HOST arrays of device pointers.
 * Weight gradients accumulate (+=) into the grad_table slots (per-sample partials, fixed-order per-modality
 * reduction: deterministic); NULL slots are skipped.
 *
 * heads: table[6*m + {0..5}] = {w1, b1, w2, b2, pw, pb} of modality_decoders.m.0 / .m.2 (conv3x3 c->c, KRSC)
 * and modality_output_projectors.m (1x1 c->1; NULL/NULL for colour modalities). rec / drec [nb][h][w][c];
 * out / dout [nb][h][w][out_c]: the projector output (1 channel) or the head's first out_c channels,
 * zero-padded to out_c channels (:283-299). */
int mvae_modality_heads_fwd(const float* rec, const long long* idx, int nb, int h, int w, int c, int nm,
                            const void* const* table, int out_c, float* out, void* stream);
int mvae_modality_heads_bwd(const float* rec, const long long* idx, int nb, int h, int w, int c, int nm,
                            const void* const* table, int out_c, const float* dout, float* drec,
                            void* const* grad_table, void* workspace, size_t ws_bytes, void* stream);
size_t mvae_modality_heads_workspace_bytes(int nb, int c);
/* input routing: routed[b] = nan_to_zero(proj_m(nan_to_zero(x[b][..][0]))) when table[2*m] (1x1 conv 1->c
 * weight, table[2*m+1] its bias) is set, else nan_to_zero(x[b][..][0..c)) (channels past cx read as 0).
 * x [nb][hw][cx], routed / drouted [nb][hw][c]; the backward produces the projector weight gradients only
 * (x is data). */
int mvae_modality_route_in_fwd(const float* x, int cx, const long long* idx, int nb, int hw, int c, int nm,
                               const void* const* table, float* routed, void* stream);
int mvae_modality_route_in_bwd(const float* x, int cx, const long long* idx, int nb, int hw, int c, int nm,
                               const void* const* table, const float* drouted, void* const* grad_table,
                               void* workspace, size_t ws_bytes, void* stream);
size_t mvae_modality_route_in_workspace_bytes(int nb, int c);

/* ConditionalVAE concat conditioning (src/models/conditional_vae.py:65-69 condition_proj = Linear(K -> c*64) + ReLU
 * + Unflatten(c, 8, 8); :107-127 create_condition_map = bilinear to (h, w), align_corners=False; :131-136
 * torch.cat([x, map], 1)). x [nb][h][w][c] NHWC, cond [nb][K], w [c*64][K], bias [c*64]; writes m = relu(pre)
 * [nb][c*64] (kept for the backward) and xcond [nb][h][w][2c]. Bit-exact with the reference's CPU path for a
 * one-hot condition (the projection is W[:, idx] + bias) and for its bilinear kernel (h + w <= 128). h, w <= 256.
 * The backward accumulates dw / dbias (beta = 1) from dxcond; dpre is scratch of nb*c*64 floats. */
int mvae_condition_concat_fwd(const float* x, const float* cond, const float* w, const float* bias, float* m,
                              float* xcond, int nb, int c, int h, int wd, int K, void* stream);
int mvae_condition_concat_bwd(const float* dxcond, const float* cond, const float* m, float* dw, float* dbias,
                              float* dpre, int nb, int c, int h, int wd, int K, void* stream);

/* DisentangledConditionalVAE's batch-coupled latent losses (src/models/disentangled_conditional_vae.py:195-206
 * partition_latent in NCHW flatten order, :305-349 modality_separation_loss over the sorted distinct ids,
 * :351-386 contrastive_loss with temperature). z [nb][c][hw] logical (cl = 1: stored NHWC), partition = flat
 * elements [off, off + d); idx [nb] int64. Forward: out[0] = separation, out[1] = contrastive, out[2] = rows with
 * positives. Backward: gsep / gcon are device scalars (upstream gradients; a non-finite forward value drops its
 * term), dz (zero-filled by the caller, same layout as z) receives the partition's gradient. nb <= 1024, d <= 16;
 * workspace from the query, shared by the forward and its backward. */
int mvae_latent_aux_fwd(const float* z, const long long* idx, int nb, int c, int hw, int cl, int off, int d,
                        float temperature, float* out, float* workspace, size_t ws_bytes, void* stream);
int mvae_latent_aux_bwd(const float* z, const long long* idx, int nb, int c, int hw, int cl, int off, int d,
                        float temperature, const float* out, const float* gsep, const float* gcon, float* dz,
                        float* workspace, size_t ws_bytes, void* stream);
size_t mvae_latent_aux_workspace_bytes(int nb, int d);

#ifdef __cplusplus
}
#endif
#endif /* MEDVAE_HIP_H */
