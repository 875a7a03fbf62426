/*
 * fen.h -- C-ABI of libfen_hip.so, the MI355X (gfx950) kernels behind the FaceEnhanceNet
 * forward/backward hot path.
 *
 * Plain C: device pointers, sizes and an opaque hipStream_t (passed as void*).  No torch
 * types.  Every entry point is asynchronous on `stream`, allocates nothing, never syncs,
 * and returns 0 (FEN_OK) or a negative fen_status.  fen_status_string() names the code.
 *
 * Activations are NHWC (channels-last) in the compute dtype (FEN_F32, FEN_BF16 or FEN_F16).
 * Weights are the reference's OIHW fp32 tensors; fen_pack_conv_w() repacks them into the
 * kernel layout [9 taps][Cout_pad][Cin] of the compute dtype.
 *
 * Each entry point replaces an aten op (or a fused chain of them) that the reference
 * calls from src/models (reference file:line given per entry); see SURVEY.md §8a/§8b.
 */
#ifndef FEN_H
#define FEN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    FEN_OK = 0,
    FEN_EINVAL = -1,        /* bad pointer / shape / alignment                  */
    FEN_EUNSUPPORTED = -2,  /* valid request outside what the kernels implement */
    FEN_EHIP = -3,          /* a HIP launch error                               */
    FEN_ERCCL = -4          /* an RCCL call failed (fen_last_rccl_error names it) */
} fen_status;

typedef enum { FEN_F32 = 0, FEN_BF16 = 1, FEN_F16 = 2 } fen_dtype;

/* conv3x3 epilogue flags (fen_conv_desc.epi) */
enum {
    FEN_EPI_BIAS = 1,       /* v += bias[co]                                                    */
    FEN_EPI_PRELU = 2,      /* y_pre = v (if y_pre); y = v>0 ? v : alpha[c]*v                   */
    FEN_EPI_SHUFFLE = 4,    /* PixelShuffle(2) store: packed rows are permuted (see pack mode 1)*/
    FEN_EPI_PRELU_BWD = 8,  /* y = v*(pre>0?1:alpha[co]); part[blk][co] = sum v*pre*(pre<=0)     */
    FEN_EPI_UNSHUFFLE = 16, /* inverse PixelShuffle(2) store: y is [B,H/2,W/2,4*Cout]           */
    FEN_EPI_POOL = 32,      /* part[b][tile][co] = sum over the tile's pixels of the stored v   */
    FEN_EPI_LAST = 64,      /* conv_last: + bicubic skip, eval clamp, NCHW fp32 out, L1 grad    */
    FEN_EPI_DOT = 128,      /* part[b][tile][co] = sum over the tile of (stored v) * pre_in      */
    FEN_EPI_RELU_BWD = 4096 /* y = pre_in>0 ? v : 0 (ReLU backward through the ReLU output pre_in;
                               no partial sums: the frozen VGG19 extractor's data gradients,
                               perceptual.py:60-64).  Not with PRELU_BWD / DOT / LAST / SHUFFLE.  */
};

/* 3x3, stride 1, pad 1 convolution as an implicit GEMM on MFMA.
 *   forward : RCAB conv1/conv2 (blocks.py:123-131,145-147), ResidualGroup conv (blocks.py:182-189),
 *             conv_after_body (custom.py:109-112,172-175), PixelShuffleUpsample conv+shuffle+PReLU
 *             (blocks.py:211-227), conv_last + bicubic skip + clamp (custom.py:121-124,158-161,181-188)
 *   backward: the same kernel is the data-gradient (dgrad) of every 3x3 conv when given
 *             fen_pack_conv_w(mode 2) weights; its epilogue fuses PReLU backward and the
 *             PixelShuffle inverse (autograd of blocks.py:146,225-226).                        */
typedef struct {
    int dtype;                 /* fen_dtype of x, w, y, y_pre, res[], pre_in                    */
    int B, H, W, Cin, Cout;    /* conv geometry (output = input spatial size)                   */
    const void* x;             /* NHWC [B,H,W,Cin]                                              */
    const void* w;             /* packed [9][Cout_pad][Cin], Cout_pad = Cout rounded up to 16    */
    const float* bias;         /* [Cout] (FEN_EPI_BIAS)                                         */
    int epi;                   /* FEN_EPI_* bitmask                                             */
    const float* alpha;        /* PReLU slopes: [Cout/4] with SHUFFLE, else [Cout]              */
    void* y;                   /* output: NHWC [B,H,W,Cout] | SHUFFLE [B,2H,2W,Cout/4] |
                                  UNSHUFFLE [B,H/2,W/2,4*Cout] | LAST NCHW fp32 [B,Cout,H,W]     */
    void* y_pre;               /* FEN_EPI_PRELU: pre-activation copy, same layout as y (or NULL) */
    const void* res[3];        /* residual tensors NHWC [B,H,W,Cout] added to v (or NULL)       */
    const void* pre_in;        /* FEN_EPI_PRELU_BWD: pre-activation NHWC [B,H,W,Cout]; FEN_EPI_DOT:
                                  the tensor dotted with the output (the next RCAB's SE input t:
                                  the SE backward's sum dy*t, blocks.py:83-92, without a pass)   */
    float* part;               /* POOL / PRELU_BWD partial sums [B*tiles][Cout], tiles=ceil(H/16)*ceil(W/16) */
    /* FEN_EPI_LAST only */
    const float* lr;           /* LR input NCHW fp32 [B,Cout,H/scale,W/scale] for the bicubic skip */
    int scale;                 /* skip scale factor (4 for 64->256)                             */
    int clamp;                 /* 1 = eval-mode clamp to [0,1]                                  */
    const float* hr;           /* target NCHW fp32 [B,Cout,H,W] or NULL (then no loss)          */
    void* dout;                /* dL/dsr in NHWC16 dtype layout [B,H,W,16] (zero padded) or NULL */
    float l1_scale;            /* dL/dsr = sign(sr-hr) * l1_scale   (weight / numel)             */
    float* loss_part;          /* [B*tiles] partial sums of |sr-hr|                              */
    int debug;                 /* 0; tuning ablations only (1: skip epilogue, 2: skip MFMA loop)  */
    /* stride-2 convs as stride-1 convs over the space-to-depth input (fen_s2d2): a 3x3 stride-2
     * conv of C channels = this conv with Cin = 4C and the filter scattered by fen_s2d_filter
     * rule, of which only (1 + a)(1 + b) taps are non-zero for input phase (a, b).  s2d_in = C:
     * skip the zero taps per input panel (forward, mode-0 pack); s2d_out = C: per output channel
     * tile (its data gradient, mode-2 pack, Cout = 4C).  0 = off.  Streamed kernel only.       */
    int s2d_in;
    int s2d_out;
    /* Training's saved pre-activation of a PReLU with positive slopes is redundant: for an
     * aligned group of 4 channels (c & ~3 .. +3) whose slopes are all > 0, v = y > 0 ? y : y/alpha.
     * pre_elide (FEN_EPI_PRELU with y_pre): the kernel MAY skip y_pre for such groups (it may
     * also write it).  post_in (FEN_EPI_PRELU_BWD): the PReLU output y, same layout as pre_in, or
     * NULL; for such groups the pre-activation is recovered from post_in and pre_in is not read,
     * every other group reads pre_in.  (The upsampler stages, blocks.py:225-226.)              */
    int pre_elide;
    const void* post_in;
    /* The 2x2 max pool of the output (the VGG19 conv -> ReLU -> 'M' layers of the perceptual
     * extractor, perceptual.py:50-53): y_pool (or NULL) = max over each 2x2 window of y, NHWC
     * [B,H/2,W/2,Cout]; needs FEN_EPI_PRELU without SHUFFLE / UNSHUFFLE / LAST / POOL / DOT and
     * H, W even.  The 16-bit persistent kernels (bias + PReLU, no residuals) fuse it into their
     * store; every other route stores y and pools it in a second launch.  y_images > 0 (needs
     * y_pool): the kernel MAY skip storing y (and y_pre) for images b >= y_images -- the target
     * half of VGG's [pred; target] batch, whose activations no backward reads; y_pool is
     * written for every image.  0: y for every image.                                         */
    void* y_pool;
    int y_images;
} fen_conv_desc;

int fen_conv3x3(const fen_conv_desc* d, void* stream);

/* Weight gradient of a 3x3 conv: dW[co][ci][kh][kw] = sum_px dy[px][co] * x[px+tap][ci],
 * db[co] = sum_px dy[px][co].  Two launches: partial slabs then a deterministic reduction.
 * (autograd of every nn.Conv2d on the hot path; trainer.py:482-485)                       */
typedef struct {
    int dtype;
    int B, H, W, Cin, Cout;    /* Cout % 16 == 0 (the dy tensor's channel count)            */
    int cout_valid;            /* rows of dW actually written (<= Cout; conv_last: 3)        */
    const void* x;             /* NHWC [B,H,W,Cin]                                          */
    const void* dy;            /* NHWC [B,H,W,Cout]                                         */
    float* dw;                 /* OIHW fp32 [cout_valid][Cin][3][3]                         */
    float* db;                 /* [cout_valid] or NULL                                      */
    int accumulate;            /* 1: dw += ..., db += ...                                   */
    float* work;               /* workspace, fen_wgrad_work_floats() floats                 */
} fen_wgrad_desc;

size_t fen_wgrad_work_floats(const fen_wgrad_desc* d);
int fen_wgrad3x3(const fen_wgrad_desc* d, void* stream);

/* n (<= FEN_WGRAD_MAXJOBS) independent weight gradients of one shape (B, H, W, Cin, Cout,
 * dtype) in one launch pair: the CUs are split between the jobs, so each block reduces n x
 * as many pixel tiles into its fp32 slab and the slabs (written and re-read) shrink n-fold.
 * One shared workspace: descs[0].work, fen_wgrad_multi_work_floats() floats (the other
 * descs' work fields are ignored).  Results equal fen_wgrad3x3 per job up to fp32
 * summation order (deterministic run to run).  The backward's conv1/conv2 weight gradients
 * of consecutive RCABs (autograd of blocks.py:135-153's convs; trainer.py:482-485).       */
#define FEN_WGRAD_MAXJOBS 32
size_t fen_wgrad_multi_work_floats(int n, const fen_wgrad_desc* descs);
int fen_wgrad3x3_multi(int n, const fen_wgrad_desc* descs, void* stream);

/* conv_first forward: NCHW fp32 [B,Ci,H,W] -> NHWC [B,H,W,C] (custom.py:91-94,164)          */
int fen_conv_first_fwd(int dtype, int B, int Ci, int H, int W, int C, const float* x,
                       const float* w, const float* bias, void* y, void* stream);
/* ... with the VGG19 input stage (perceptual.py:67-72,84-95): in-bounds samples become
 * (x - in_mean[ci]) * in_istd[ci] before the zero padding (in_mean / in_istd may be NULL:
 * identity); act >= 0 applies a leaky ReLU of slope act to y (0: ReLU; 0.2: the
 * discriminator's first block, discriminator.py:47-55), act < 0 none.                     */
int fen_conv_first_fwd_ex(int dtype, int B, int Ci, int H, int W, int C, const float* x,
                          const float* w, const float* bias, const float* in_mean, const float* in_istd,
                          float act, void* y, void* stream);
/* conv_first weight gradient (no data gradient: x needs none) -> dw OIHW, db              */
size_t fen_conv_first_work_floats(int B, int Ci, int H, int W, int C);
int fen_conv_first_wgrad(int dtype, int B, int Ci, int H, int W, int C, const float* x,
                         const void* dy, float* dw, float* db, int accumulate, float* work,
                         void* stream);

/* conv_last data gradient fused with the previous stage's PReLU backward and the
 * PixelShuffle inverse: dout NHWC16 [B,H,W,16] -> du NHWC [B,H/2,W/2,4C];
 * pre = that stage's pre-activation NHWC [B,H,W,C]; part[rows][C] dalpha partials.
 * post = that stage's PReLU output (same layout) or NULL: as fen_conv_desc.post_in, groups of
 * 4 channels with all slopes > 0 recover the pre-activation from it and do not read pre.
 * part has fen_conv_last_dgrad_part_rows rows (one per block of the persistent grid; the
 * slope gradient is their column sum).                                                     */
size_t fen_conv_last_dgrad_part_rows(int B, int H, int W);
int fen_conv_last_dgrad(int dtype, int B, int H, int W, int C, int Co, const void* dout,
                        const float* w, const void* pre, const void* post, const float* alpha,
                        void* du, float* part, void* stream);
/* conv_last's whole backward in one pass (replaces the conv_last weight-gradient pass + the
 * call above on the training path; custom.py:177-184 backward): du and the slope partials as
 * fen_conv_last_dgrad, plus dw_part[rows][Co*C*9] (OIHW order) and db_part[rows][Co], whose
 * column sums are conv_last's weight and bias gradients; rows = fen_conv_last_dgrad_part_rows.
 * post is required (the stage's PReLU output is the weight gradient's operand).  16-bit, C = 64,
 * Co <= 3, H and W multiples of 16 (fen_conv_last_bwd_supported); FEN_EUNSUPPORTED otherwise. */
int fen_conv_last_bwd_supported(int dtype, int B, int H, int W, int C, int Co);
int fen_conv_last_bwd(int dtype, int B, int H, int W, int C, int Co, const void* dout,
                      const float* w, const void* pre, const void* post, const float* alpha,
                      void* du, float* dal_part, float* dw_part, float* db_part, void* stream);

/* Channel attention (blocks.py:44-92) forward: pool partials -> s = sigmoid(W2 relu(W1 mean)) */
int fen_se_fwd(int B, int C, int Cr, int nparts, float inv_hw, const float* part,
               const float* w1, const float* w2, float* mean, float* hid, float* s, void* stream);
/* SE gate and apply in one launch (replaces fen_se_fwd + fen_se_apply on the forward path;
 * ChannelAttention.forward blocks.py:83-92 and RCAB's `out * res_scale + x`, blocks.py:149-153):
 * y = t * s[b,c] * res_scale + x with s computed from the pool partials as in fen_se_fwd.
 * mean / hid / s (optional, may be NULL) receive the gate's intermediates.                   */
int fen_se_fused(int dtype, int B, int HW, int C, int Cr, int nparts, float inv_hw, const float* part,
                 const float* w1, const float* w2, float* mean, float* hid, float* s, const void* t,
                 float res_scale, const void* x, void* y, void* stream);
/* y = t * s[b,c] * res_scale + x   (blocks.py:92,153)                                       */
int fen_se_apply(int dtype, int B, int HW, int C, const void* t, const float* s, float res_scale,
                 const void* x, void* y, void* stream);
/* part[b][chunk][c] = sum over the chunk's pixels of a*b_ (b_ may be NULL -> sum of a)     */
size_t fen_pool_parts(int HW);
int fen_pool_dot(int dtype, int B, int HW, int C, const void* a, const void* b_, float* part,
                 void* stream);
/* SE backward (per image): ds = rs*sum(dy*t) -> sigmoid/FC/ReLU/FC backward.
 * g[b][c] = dL/dmean / HW; dw1p[b][Cr][C], dw2p[b][C][Cr] per-image weight-grad partials. */
int fen_se_bwd(int B, int C, int Cr, int nparts, float inv_hw, float res_scale,
               const float* part, const float* mean, const float* hid, const float* s,
               const float* w1, const float* w2, float* g, float* dw1p, float* dw2p, void* stream);
/* fen_se_bwd + fen_se_bwd_apply in one launch (same arithmetic, same results): every block
 * recomputes its image's SE backward from the pool_dot partials and writes its slice of
 * dt = dy * res_scale * s[b,c] + g[b,c]; g (may be NULL), dw1p, dw2p as fen_se_bwd.
 * C <= 64, nparts <= 64, C * Cr <= 4096 (else FEN_EUNSUPPORTED: use the pair).             */
int fen_se_bwd_fused(int dtype, int B, int HW, int C, int Cr, int nparts, float inv_hw, float res_scale,
                     const float* part, const float* mean, const float* hid, const float* s,
                     const float* w1, const float* w2, const void* dy, float* g, float* dw1p, float* dw2p,
                     void* dt, void* stream);
/* dt = dy * s[b,c] * res_scale + g[b,c]                                                    */
int fen_se_bwd_apply(int dtype, int B, int HW, int C, const void* dy, const float* s,
                     float res_scale, const float* g, void* dt, void* stream);


/* RCAB with the SE gate deferred to the consumer (blocks.py:135-153 + ChannelAttention
 * blocks.py:83-92, one launch per RCAB of a ResidualGroup's chain, blocks.py:185-188).
 * The gate of RCAB j needs the global mean of its t_j, i.e. every tile of the image; instead
 * of a grid-wide hand-off inside the launch, launch j+1 applies it while it builds its input:
 *     x_j = x_{j-1} + res_scale * s_{j-1} * t_{j-1}      (s_{j-1} from part_{j-1}, fc*_{j-1})
 *     z1 = conv1(x_j)+b1, a1 = PReLU(z1), t_j = conv2(a1)+b2, part_j = per-tile sums of t_j.
 * Chain start (tp == NULL): x_j = x (no gate).  Chain end: fen_se_fused(part, t, x) gives
 * the group's last RCAB output.  Every block is independent (no in-launch synchronisation, any
 * grid, graph-replayable, no workspace).  16-bit (bf16 / fp16) NHWC, C = 64, Cr <= 16, H and
 * W multiples of 16.  part layout [B][H*W/256][64] (fen_se_fused's nparts = H*W/256).        */
typedef struct {
    int dtype;                 /* FEN_BF16 or FEN_F16                                          */
    int B, H, W, C, Cr;
    const void* x;             /* x_{j-1} (deferred) or x_j (chain start), NHWC [B,H,W,64]     */
    const void* tp;            /* t_{j-1} NHWC, or NULL at the chain start                     */
    const float* pp;           /* part_{j-1} [B][tiles][64]                                    */
    const float* pfc1;         /* RCAB j-1 channel_attention.fc.0.weight [Cr][64]              */
    const float* pfc2;         /* RCAB j-1 channel_attention.fc.2.weight [64][Cr]              */
    float res_scale;           /* 0.2                                                          */
    float inv_hw;              /* 1/(H*W)                                                      */
    float* ps;                 /* s_{j-1} [B][64] user copy (or NULL; written by tile 0 of b)  */
    float* pmean;              /* mean_{j-1} [B][64] (or NULL)                                 */
    float* phid;               /* hid_{j-1} [B][Cr] (or NULL)                                  */
    void* xo;                  /* x_j out NHWC (deferred mode; NULL allowed only at the start) */
    const void* w1;            /* conv1 packed mode 0 [9][64][64]                              */
    const float* b1;
    const float* alpha;        /* PReLU [64]                                                   */
    const void* w2;            /* conv2 packed mode 0                                          */
    const float* b2;
    void* t;                   /* t_j out NHWC                                                 */
    float* part;               /* part_j out [B][tiles][64]                                    */
    void* z1;                  /* training copies (or NULL): conv1 pre-activation and PReLU    */
    void* a1;
    unsigned long long* stamps;/* NULL; diagnostic build only (-DFEN_STAMPS): phase timestamps */
} fen_rcab_deferred_desc;
int fen_rcab_deferred_supported(int dtype, int B, int H, int W, int C, int Cr);
int fen_rcab_deferred(const fen_rcab_deferred_desc* d, void* stream);

/* A ResidualGroup's end in one launch (blocks.py:185-189): the last RCAB's gate and scaled
 * residual, y = x + res_scale * s * t, applied while building the input (d describes that
 * RCAB exactly as for a deferred launch: x, tp, pp, pfc1, pfc2, res_scale, inv_hw, the
 * optional ps / pmean / phid copies, and xo = y out or NULL), then the group conv
 * out = conv(y; w packed mode 0, bias) + res (the group's input).  d's conv fields are
 * ignored.  Replaces fen_se_fused + fen_conv3x3 at the chain end.                          */
int fen_rcab_group_end(const fen_rcab_deferred_desc* d, const void* w, const float* bias, const void* res,
                       void* out, void* stream);

/* A whole ResidualGroup in ONE persistent launch (ResidualGroup.forward, blocks.py:185-189:
 * nb x RCAB.forward blocks.py:135-153 with ChannelAttention blocks.py:83-92, then the group
 * conv and the group's skip), inference, or training with `save` (the backward's saved
 * tensors written as the chain runs).  Each image is cut into H/8 strips of 8 rows x 64
 * columns; one block (one CU) keeps its strip resident (x_j in registers, x_j / a1 and the
 * running conv's filter in LDS) for all nb RCABs; the strips of an image exchange only the SE
 * pool partials and their first / last rows (sc1 hand-offs through `work`).  y may not alias x.
 * 16-bit NHWC, C = 64, W = 64, H a multiple of 8 (<= 128), Cr <= 16, nb <= FEN_GS_MAXNB.
 * `work`: fen_group_strip_work_bytes(B, H) bytes, ZEROED once before the first launch; the
 * kernel leaves its counters at zero (graph-replayable), and sets the int at byte 8 to nonzero
 * if a hand-off wait timed out (then the output is invalid).  Grid = B * H/8 blocks, taken in
 * start order (no co-residency assumption).                                                 */
#define FEN_GS_MAXNB 20
typedef struct {
    int dtype;                 /* FEN_BF16 or FEN_F16                                          */
    int B, H, W, C, Cr, nb;
    float res_scale;           /* 0.2                                                          */
    const void* x;             /* group input NHWC [B,H,64,64]                                 */
    void* y;                   /* group output NHWC (conv(chain(x)) + bias + x)                */
    const void* w1[FEN_GS_MAXNB];      /* per RCAB: conv1 packed mode 0 [9][64][64]           */
    const float* b1[FEN_GS_MAXNB];
    const float* alpha[FEN_GS_MAXNB];  /* PReLU [64]                                           */
    const void* w2[FEN_GS_MAXNB];      /* conv2 packed mode 0                                  */
    const float* b2[FEN_GS_MAXNB];
    const float* fc1[FEN_GS_MAXNB];    /* channel_attention.fc.0.weight [Cr][64]               */
    const float* fc2[FEN_GS_MAXNB];    /* channel_attention.fc.2.weight [64][Cr]               */
    float* s_out[FEN_GS_MAXNB];        /* optional: each RCAB's gate s [B][64] (or NULL)       */
    const void* wg;            /* the group conv, packed mode 0                                */
    const float* bg;
    void* work;
    size_t work_bytes;
    /* training (save = 1): the backward's operands, written as the chain runs (NHWC, 16-bit,
     * [B,H,64,64]; x_j = RCAB j's input: sv_x[0] is not written, the group input x is it) */
    int save;
    void* sv_x[FEN_GS_MAXNB];
    void* sv_z1[FEN_GS_MAXNB];         /* conv1 + b1, before PReLU                             */
    void* sv_a1[FEN_GS_MAXNB];         /* PReLU(z1)                                            */
    void* sv_t[FEN_GS_MAXNB];          /* conv2 + b2                                           */
    float* sv_mean[FEN_GS_MAXNB];      /* the SE pool means [B][64]                            */
    float* sv_hid[FEN_GS_MAXNB];       /* ReLU(FC1(mean)) [B][Cr]  (s goes to s_out)           */
    void* x_last;                      /* the chain's output = the group conv's input          */
    /* optional (NULL = off): where a timed-out hand-off wait is reported.  The launch's last
     * block stores FEN_STATUS_GS_FWD there (a system-scope store: host-mapped pinned memory
     * may be passed, read by the host without a sync) and clears the workspace's error word;
     * the word is never cleared by the kernel -- the caller resets it after reading.  With
     * status NULL the error word stays set in `work` (byte 8) instead.                        */
    int* status;
    int fault;                         /* test-only fault injection: nonzero = the block with
                                          ticket 1 skips RCAB 0's a1 flag (its neighbour's wait
                                          times out after ~1 s); 0 in production              */
    /* training: sv_z1[j] is not written when every slope alpha[j][c] is > 0 (z1 = a1 > 0 ? a1 :
     * a1 / alpha then; fen_group_strip_bwd given a1 recovers it); 0 = always written          */
    int pre_elide;
} fen_group_strip_desc;
#define FEN_STATUS_GS_FWD 1            /* a fen_group_strip wait timed out (output invalid)     */
#define FEN_STATUS_GS_BWD 2            /* a fen_group_strip_bwd wait timed out                  */
#define FEN_STATUS_GS_TABLE 4          /* a fen_group_strip_chain launch found no prepared table for
                                          its descriptors in `work`: it computed nothing           */
int fen_group_strip_supported(int dtype, int B, int H, int W, int C, int Cr, int nb);
size_t fen_group_strip_work_bytes(int B, int H);
int fen_group_strip(const fen_group_strip_desc* d, void* stream);
/* ng consecutive ResidualGroups (reference custom.py:168-169, the body's group loop) as ONE
 * launch: d[0..ng-1] are the groups' descriptors as for fen_group_strip (all with the same
 * save and pre_elide: training writes every group's saved set as fen_group_strip does),
 * d[g].y == d[g+1].x, all sharing d[0].work (fen_group_strip_chain_work_bytes(B, H, ng) bytes:
 * the workspace plus the groups' parameter table), d[0].status / fault used.  A strip stays on
 * its CU across the groups: group g's output rows become group g+1's x_0 in registers, the
 * neighbours' boundary rows by hand-off; each group's output is still written to d[g].y (the
 * next group's skip input).  fen_group_strip_chain_prepare writes the parameter table into
 * `work` (fen_group_strip_chain_work_bytes(B, H, ng) bytes: the workspace, a 256-B header, the
 * rows), asynchronously on `stream` (kernel-argument copies: no host sync, no host buffer kept,
 * capturable); prepare once per (descriptors, work) before the launches that use them, again
 * after `work` is (re)allocated.  The launch hashes its own descriptors; every block compares
 * that with the header before it reads a row, and on a mismatch (never prepared, prepared for
 * other descriptors, a fresh buffer) the launch computes nothing and reports
 * FEN_STATUS_GS_TABLE through d[0].status (else the workspace's error word, byte 8, bit 1).
 * (ng + 1) * (nb + 1) <= 254.                                                                 */
/* optional: the body's conv_after_body (custom.py:172-175: conv(body output) + bias + feat0) as
 * a last "group" of no RCABs in the same launch; its input is d[ng-1].y                        */
typedef struct {
    const void* w;             /* conv_after_body packed mode 0 [9][64][64]                    */
    const float* bias;         /* [64]                                                         */
    const void* skip;          /* the residual added: the body's input (feat0)                 */
    void* y;                   /* out NHWC [B,H,64,64] (not d[ng-1].y, not skip)               */
} fen_group_strip_chain_tail;
size_t fen_group_strip_chain_work_bytes(int B, int H, int ng);   /* room for ng groups + a tail */
int fen_group_strip_chain_prepare(const fen_group_strip_desc* d, int ng, const fen_group_strip_chain_tail* tail,
                                  void* stream);
int fen_group_strip_chain(const fen_group_strip_desc* d, int ng, const fen_group_strip_chain_tail* tail, void* stream);

/* 128-channel RCAB convs (BASELINE configs[4]: num_channels = 128, Cr = 32; RCAB blocks.py:
 * 135-153, ChannelAttention blocks.py:83-92, ResidualGroup blocks.py:185-189), one launch per
 * conv with the RCAB's elementwise work folded in; replaces the per-op conv + fen_se_fused
 * launches at C = 128.  With tp != NULL the input is built with the previous RCAB's gate
 * (deferred as in fen_rcab_deferred): in = x + res_scale * s * tp, s from pp / pfc1 / pfc2
 * (its per-image copy to ps when ps != NULL), in's own tiles to xo when xo != NULL.
 *   mode 1 (conv1):      y = PReLU(conv(in) + bias; alpha)   (z1 = conv(in) + bias if z1 != NULL)
 *   mode 2 (conv2):      y = conv(x) + bias; part = per-tile channel sums of y (fp32, before the
 *                        16-bit rounding) [B][fen_rcab_c128_tiles(H, W)][128]  (tp must be NULL)
 *   mode 3 (group conv): y = conv(in) + bias + res
 *   mode 4 (upsampler stage): y = PReLU(PixelShuffle(2)(conv(x) + bias); alpha), y [B,2H,2W,128];
 *                        w = the conv(128 -> 512) packed mode 1 [9][512][128] (shuffle-permuted
 *                        rows), bias [512], alpha [128]  (tp must be NULL)
 * 16-bit NHWC [B,H,W,128]; H % 4 == 0, W % 64 == 0, Cr <= 32; w packed mode 0 [9][128][128]
 * (mode 4: as stated there).
 * Every block is independent (any grid, graph-replayable, no workspace).  y may not alias x,
 * tp; xo may not alias x, tp.                                                                   */
typedef struct {
    int dtype;                 /* FEN_BF16 or FEN_F16                                          */
    int B, H, W, C, Cr;
    int mode;                  /* 1 .. 4 as above                                              */
    float res_scale;           /* 0.2                                                          */
    const void* x;             /* the conv input, or x_{j-1} with tp                           */
    const void* tp;            /* t_{j-1} (deferred gate) or NULL                              */
    const float* pp;           /* part of t_{j-1} (a mode-2 launch's)                          */
    const float* pfc1;         /* RCAB j-1 channel_attention.fc.0.weight [Cr][128]             */
    const float* pfc2;         /* RCAB j-1 channel_attention.fc.2.weight [128][Cr]             */
    float* ps;                 /* s_{j-1} [B][128] copy or NULL                                */
    void* xo;                  /* x_j = x + res_scale * s * tp out, or NULL                    */
    const void* w;             /* packed mode 0                                                */
    const float* bias;
    const float* alpha;        /* mode 1: PReLU [128]                                          */
    const void* res;           /* mode 3: the residual (the group's input)                     */
    void* y;
    void* z1;                  /* mode 1: optional pre-activation copy                         */
    float* part;               /* mode 2                                                       */
} fen_rcab_c128_desc;
int fen_rcab_c128_supported(int dtype, int B, int H, int W, int C, int Cr);
int fen_rcab_c128_tiles(int H, int W);
int fen_rcab_c128(const fen_rcab_c128_desc* d, void* stream);

/* The backward of a whole ResidualGroup in ONE persistent launch (autograd of
 * ResidualGroup.forward blocks.py:185-189 and of each RCAB blocks.py:135-153 /
 * ChannelAttention blocks.py:83-92), on the saved tensors of a training fen_group_strip:
 *   d = conv_g^T(dy);  for j = nb-1 .. 0:  SE backward (a = sum over the image of d * t_j),
 *   dt_j = d * res_scale * s_j + g_j,  dz1_j = conv2_j^T(dt_j) * PReLU'(z1_j),
 *   d += conv1_j^T(dz1_j);  dx = d + dy (+ dres).
 * Writes dt_j and dz1_j (the conv2 / conv1 weight gradients' dy operands: run
 * fen_wgrad3x3_multi on (a1_j, dt_j), (x_j, dz1_j) and (x_last, dy) afterwards),
 * dalpha_part_j [fen_group_strip_bwd_dal_rows(B, H)][64] (sum over each strip of 8 image rows of
 * conv2^T(dt) * z1 * [z1 <= 0], rows in order: column sums give prelu.weight's gradient), dw1p_j [B][Cr][64] and dw2p_j [B][64][Cr] (per-image SE weight
 * gradients: column sums over B).  Same strips, envelope and hand-off scheme as
 * fen_group_strip (its own `work`, fen_group_strip_bwd_work_bytes, ZEROED once).  w*t / wgt are
 * the mode-2 (transposed) packs.  dx may not alias dy or dres.                                */
typedef struct {
    int dtype;                 /* FEN_BF16 or FEN_F16                                          */
    int B, H, W, C, Cr, nb;
    float res_scale;
    const void* dy;            /* the group output's gradient NHWC [B,H,64,64]                 */
    void* dx;                  /* the group input's gradient                                   */
    const void* dres;          /* optional second residual gradient added to dx (or NULL)      */
    const void* wgt;           /* the group conv, packed mode 2                                */
    const void* w1t[FEN_GS_MAXNB];     /* per RCAB: conv1 packed mode 2                        */
    const void* w2t[FEN_GS_MAXNB];     /* conv2 packed mode 2                                  */
    const float* alpha[FEN_GS_MAXNB];
    const float* fc1[FEN_GS_MAXNB];    /* [Cr][64]                                             */
    const float* fc2[FEN_GS_MAXNB];    /* [64][Cr]                                             */
    const void* z1[FEN_GS_MAXNB];      /* saved: conv1 + b1                                    */
    const void* t[FEN_GS_MAXNB];       /* saved: conv2 + b2                                    */
    const float* s[FEN_GS_MAXNB];      /* saved gates [B][64]                                  */
    const float* mean[FEN_GS_MAXNB];   /* saved pool means [B][64]                             */
    const float* hid[FEN_GS_MAXNB];    /* saved ReLU(FC1(mean)) [B][Cr]                        */
    void* dt[FEN_GS_MAXNB];            /* out: dL/dt NHWC                                      */
    void* dz1[FEN_GS_MAXNB];           /* out: dL/dz1 NHWC                                     */
    float* dalpha_part[FEN_GS_MAXNB];  /* out: [B*H/8][64], one row per strip                   */
    float* dw1p[FEN_GS_MAXNB];         /* out: [B][Cr][64]                                     */
    float* dw2p[FEN_GS_MAXNB];         /* out: [B][64][Cr]                                     */
    void* work;
    size_t work_bytes;
    int* status;                       /* as fen_group_strip_desc.status (FEN_STATUS_GS_BWD)   */
    int fault;                         /* test-only: ticket 1 skips the first RCAB's dz1 flag  */
    /* optional (NULL = off): the saved a1 = PReLU(z1); for an RCAB whose slopes are all > 0 the
     * pre-activation is recovered from it (a1 > 0 ? a1 : a1 / alpha) and z1[j] is not read --
     * the forward's pre_elide                                                                */
    const void* a1[FEN_GS_MAXNB];
} fen_group_strip_bwd_desc;
int fen_group_strip_bwd_supported(int dtype, int B, int H, int W, int C, int Cr, int nb);
size_t fen_group_strip_bwd_work_bytes(int B, int H);
int fen_group_strip_bwd_dal_rows(int B, int H);      /* rows of each dalpha_part_j: B * H / 8 */
int fen_group_strip_bwd(const fen_group_strip_bwd_desc* d, void* stream);

/* The RCAB backward's two data gradients in one launch (autograd of blocks.py:145-147):
 *   dz1 = conv2^T(dt) * PReLU'(z1),  dalpha_part[b][tile][c] = sum over the tile of
 *   conv2^T(dt) * z1 * (z1 <= 0),  dx = conv1^T(dz1) + dy,
 *   optionally dot_part[b][tile][c] = sum over the tile of dx (as stored) * dot_t.
 * dt is the SE backward's output, w2t / w1t the conv2 / conv1 mode-2 packs (no bias), z1
 * the saved pre-activation.  The same persistent tile pipeline as fen_rcab_deferred (dz1
 * recomputed on each tile's 18x18 halo); the envelope of fen_rcab_deferred_supported.     */
typedef struct {
    int dtype;                 /* FEN_BF16 or FEN_F16                                          */
    int B, H, W, C;            /* C = 64                                                        */
    const void* dt;            /* NHWC [B,H,W,64]                                               */
    const void* w2t;           /* conv2 packed mode 2                                           */
    const void* z1;            /* conv1 pre-activation NHWC                                     */
    const float* alpha;        /* PReLU slopes [64]                                             */
    const void* w1t;           /* conv1 packed mode 2                                           */
    const void* dy;            /* the RCAB's output gradient, added to dx (the residual path)   */
    void* dz1;                 /* out NHWC (conv1's weight-gradient operand)                    */
    float* dalpha_part;        /* out [B*tiles][64]                                             */
    void* dx;                  /* out NHWC                                                      */
    const void* dot_t;         /* NULL or NHWC: the next RCAB's t (with dot_part)                */
    float* dot_part;           /* NULL or out [B*tiles][64]                                     */
    /* The SE backward folded in (se_part != NULL; else these are ignored): dt is then an OUTPUT,
     * dt = dy * se_res_scale * s + g with fen_se_bwd_fused's arithmetic (g from the FC chain
     * over se_part), built on each tile's dy halo in LDS; the FC weight-gradient rows go to
     * se_dw1p / se_dw2p exactly as fen_se_bwd_fused writes them.  <= 6 tiles per CU and <= 64
     * tiles per image.  Replaces fen_se_bwd_fused + this launch (blocks.py:88-92,150-153).    */
    const float* se_part;      /* sum over each tile of dy * t [B][tiles][64] (nparts = tiles)  */
    const float* se_s;         /* saved gate s [B][64]                                           */
    const float* se_mean;      /* saved pooled mean [B][64]                                      */
    const float* se_hid;       /* saved hidden activations [B][Cr]                               */
    const float* se_w1;        /* channel_attention.fc.0.weight [Cr][64]                         */
    const float* se_w2;        /* channel_attention.fc.2.weight [64][Cr]                         */
    float* se_dw1p;            /* out [B][Cr*64]                                                 */
    float* se_dw2p;            /* out [B][64*Cr]                                                 */
    float se_res_scale;        /* 0.2                                                            */
    int se_Cr;                 /* <= 16                                                          */
    const void* dres;          /* NULL or NHWC: a second residual added to dx (a ResidualGroup's
                                  first RCAB: the group's output gradient); not with dot_t        */
} fen_rcab_bwd_desc;
int fen_rcab_bwd(const fen_rcab_bwd_desc* d, void* stream);
/* 1 when fen_rcab_bwd takes the folded SE backward (se_part) at this shape, else 0            */
int fen_rcab_bwd_se_supported(int dtype, int B, int H, int W, int C, int Cr);

/* trainer.py:416-421 LR synthesis: bicubic x0.25, align_corners=False, NCHW fp32          */
int fen_bicubic_down4(int B, int C, int H, int W, const float* hr, float* lr, void* stream);

/* out[c] = (accumulate ? out[c] : 0) + scale * sum_r part[r][c]   (fixed-order, deterministic;
 * the per-channel reductions behind PReLU / SE-FC weight gradients and the L1 loss value)   */
int fen_colsum(int rows, int cols, const float* part, float scale, float* out, int accumulate,
               void* stream);
typedef struct {
    const float* part;
    float* out;
    int rows, cols;
    float scale;
    int accumulate;
} fen_colsum_job;
/* up to 40 independent column sums in one launch                                            */
int fen_colsum_multi(int njobs, const fen_colsum_job* jobs, void* stream);

/* OIHW fp32 -> kernel layout of dtype.  mode 0: [9][Cout_pad][Cin] rows = co;
 * mode 1: same with rows permuted for FEN_EPI_SHUFFLE (row t*Cout/4+c <- co = 4c+t);
 * mode 2: dgrad weights [9][Cin_pad][Cout], flipped taps (row = ci).                        */
int fen_pack_conv_w(int dtype, int mode, int Cout, int Cin, const float* w, void* out, void* stream);
size_t fen_packed_elems(int mode, int Cout, int Cin);
/* Many packs in one launch (the re-pack after every optimizer step).  fen_pack_table fills a
 * host buffer of fen_pack_table_bytes(njobs) bytes (job table + element offsets, *total =
 * the launch's index space: each job's packed elements rounded up to 256); the caller copies it to device memory once and replays fen_pack_multi. */
typedef struct {
    const float* w;   /* OIHW fp32 source                                                     */
    void* out;        /* packed destination of dtype                                          */
    int mode, Cout, Cin;
} fen_pack_job;
size_t fen_pack_table_bytes(int njobs);
int fen_pack_table(int dtype, int njobs, const fen_pack_job* jobs, void* table_host, size_t* total);
int fen_pack_multi(int dtype, int njobs, const void* table_dev, size_t total, void* stream);

/* fp32 <-> dtype layout conversions (NCHW fp32 <-> NHWC dtype).  nchw_to_nhwc writes
 * Cpad >= C channels per pixel, zero-filling c >= C (Cpad = 16 builds conv_last's dout).    */
int fen_nchw_to_nhwc(int dtype, int B, int C, int H, int W, int Cpad, const float* x, void* y, void* stream);
int fen_nhwc_to_nchw(int dtype, int B, int C, int H, int W, const void* x, float* y, void* stream);

/* Standalone PReLU backward + PixelShuffle inverse (UpsampleModule used on its own,
 * blocks.py:223-227): dy, pre NHWC [B,H,W,C] -> du NHWC [B,H/2,W/2,4C];
 * part[B*tiles(H,W)][C] dalpha partials.                                                    */
int fen_prelu_bwd_unshuffle(int dtype, int B, int H, int W, int C, const void* dy, const void* pre,
                            const float* alpha, void* du, float* part, void* stream);

/* clip_grad_norm_ + AdamW (trainer.py:490-503) over one flat fp32 arena.
 * fen_sumsq: part[i] partial sums of g^2 (nparts = fen_sumsq_parts(n)).
 * fen_optim_prepare: one block; reads part, writes scal[0..7]:
 *   scal[0]=grad norm, scal[1]=clip coef, scal[2]=step (incremented), scal[3]=lr,
 *   scal[4]=1-lr*wd, scal[5]=step_size=lr/bc1, scal[6]=1/sqrt(bc2)   (scal[3] is an input)
 * fen_adamw: p,m,v updated in place with g*scal[1].                                         */
int fen_sumsq_parts(size_t n);
int fen_sumsq(size_t n, const float* g, float* part, void* stream);
int fen_optim_prepare(int nparts, const float* part, float max_norm, float beta1, float beta2,
                      float wd, float* scal, void* stream);
int fen_adamw(size_t n, float* p, const float* g, float* m, float* v, const float* scal,
              float beta1, float beta2, float eps, void* stream);
/* y[i] *= s  (DP gradient averaging helper)                                                 */
int fen_scale(size_t n, float* y, float s, void* stream);
/* torch.optim.AdamW.step (amsgrad / maximize off) over up to 48 separate fp32 tensors in two
 * launches -- the discriminator's optimizer_d (reference trainer.py:230-250, 446-451): per
 * tensor p, its gradient g, exp_avg m, exp_avg_sq v (n elements each) and a device step count
 * (torch's capturable state, incremented first).  p = p (1 - lr wd) - lr / (1 - b1^t) m' /
 * (sqrt(v') / sqrt(1 - b2^t) + eps), m' = lerp(m, g, 1 - b1), v' = b2 v + (1 - b2) g^2; 1 - b1
 * and 1 - b2 passed as the caller rounds them (torch: float(1 - beta) of the Python doubles).  */
typedef struct {
    float* p;
    const float* g;
    float* m;
    float* v;
    float* step;
    size_t n;
} fen_adamw_job;
int fen_adamw_multi(int njobs, const fen_adamw_job* jobs, float lr, float beta1, float beta2, float one_minus_beta1,
                    float one_minus_beta2, float eps, float weight_decay, void* stream);

/* ---- VGG19 perceptual loss (src/losses/perceptual.py:13-169), frozen feature extractor ----
 * The convs run on fen_conv3x3 (ReLU = FEN_EPI_PRELU with zero slopes; its backward =
 * FEN_EPI_PRELU_BWD with zero slopes and pre_in = the ReLU output).  Below: the pool and the
 * loss.  NHWC of dtype, C a multiple of 8, H and W even.                                   */
/* y = max_pool2d(x, 2, 2) (torchvision vgg19.features 'M')                                  */
int fen_maxpool2(int dtype, int B, int H, int W, int C, const void* x, void* y, void* stream);
/* dx [B,H,W,C] = max-pool backward of dy [B,H/2,W/2,C] through a [B,H,W,C] (first maximum
 * of each window, torch's choice) times the ReLU mask [a > 0]; every dx element written     */
int fen_maxpool2_bwd_relu(int dtype, int B, int H, int W, int C, const void* dy, const void* a, void* dx,
                          void* stream);
/* f holds [pred; target] (n elements each): part[fen_feat_loss_parts()] = per-block sums of
 * |p - t| (l2 = 0: nn.L1Loss) or (p - t)^2 (l2 = 1: nn.MSELoss); g (n elements) =
 * (accumulate ? g : 0) + scale * d/dp (sign(p - t) or 2 (p - t)); scale = weight / n.       */
int fen_feat_loss_parts(void);
/* mean |pred - target| over n fp32 elements (nn.L1Loss, losses/combined.py:38-47): part
 * [fen_feat_loss_parts()] = per-block sums of |p - t| (fen_colsum with scale 1/n gives the loss);
 * grad (NULL: none) = scale * (gscale ? *gscale : 1) * sign(p - t), gscale a device scalar (the
 * upstream gradient of the loss: no host sync).                                              */
int fen_l1_loss(size_t n, const float* pred, const float* target, const float* gscale, float scale, float* grad,
                float* part, void* stream);
int fen_feat_loss(int dtype, size_t n, const void* f, int l2, float scale, void* g, int accumulate, float* part,
                  void* stream);

/* ---- SSIM (src/losses/ssim_loss.py:44-98, SSIMLoss 174-226; val metric trainer.py:630-634) ----
 * pred / target NCHW fp32 [B,C,H,W]; window1d = the normalised 11-tap Gaussian (2-D window =
 * its outer product, zero padding); C1 = (K1 range)^2, C2 = (K2 range)^2.
 * part[fen_ssim_parts()] (rows = C x tiles, cols = B: part[(c*ntile + tile)*B + b]) = sums of
 * the SSIM map per tile (fen_colsum over the rows gives per-image sums).  grad_mode 1: grad =
 * NCHW fp32 grad_scale * d(sum S)/d(pred) (written); 2: grad = NHWC [B,H,W,16] of dtype,
 * grad_scale * d(sum S)/d(pred) ADDED to channel c (the generator's dL/dsr buffer); 0: none. */
size_t fen_ssim_parts(int B, int C, int H, int W);
int fen_ssim(int dtype, int B, int C, int H, int W, const float* pred, const float* target, const float* window1d,
             int window_size, float C1, float C2, float* part, void* grad, float grad_scale, int grad_mode,
             void* stream);
/* The same with a workspace of fen_ssim_work_floats() floats: grad_mode 2 (C <= 3, fp32 / bf16
 * gradient buffer) runs as two launches -- the map, its tile sums and the per-pixel gradient
 * coefficients a, b, c to the workspace (fp32 for an fp32 gradient: results bit-identical to
 * the one-launch form's; fp16 for a bf16 gradient: within one bf16 ulp of them), then their
 * Gaussian filtering into the gradient; any other case (or work = NULL) is fen_ssim.  fp16
 * coefficients only while they stay inside fp16's range: |a|, |b|, |c| <= 8/C2 + 1/sqrt(C1)
 * for pixel values in [-1.5, 2.5], so a bf16 gradient takes fp32 coefficients when that
 * exceeds 16384 (C2 below ~5e-4 -- the default (0.03)^2 = 9e-4 keeps fp16). */
size_t fen_ssim_work_floats(int B, int C, int H, int W);
int fen_ssim_ex(int dtype, int B, int C, int H, int W, const float* pred, const float* target,
                const float* window1d, int window_size, float C1, float C2, float* part, void* grad,
                float grad_scale, int grad_mode, float* work, void* stream);

/* ---- HR batch preparation (src/data/transforms.py:173-279 + to_tensor 260-279) ----
 * src_u8: B uint8 HWC crops [B,P,P,3] (RGB, P even); params: B records {int flip, int
 * jitter, float brightness, contrast, saturation, int rot90_k} drawn by the host; sums: int64
 * [B] scratch; out: NCHW fp32 [B,3,P,P] = flip -> rot90 -> jitter (brightness, contrast about
 * the image mean, uint8 quantisation, 8-bit HSV saturation round trip) -> / 255.          */
int fen_augment_u8(int B, int P, const void* src_u8, const void* params, long long* sums, float* out,
                   void* stream);

/* ---- VGG-style discriminator (src/models/discriminator.py:12-219) ----
 * train-mode BatchNorm2d + LeakyReLU over NHWC [npx][C] (C % 8 == 0):
 * fen_bn_stats: stat[2C] = (mean, rstd) of y, running stats (momentum, unbiased var) updated
 * when rmean/rvar != NULL; work = fen_bn_work_floats(C) floats.
 * fen_bn_apply: out = lrelu((y - mean) * rstd * gamma + beta, slope) (eval: running stats).
 * fen_bn_bwd: dy from da for out = lrelu(BN_train(y)); dgamma / dbeta set or accumulated.
 * The _n forms run ng groups of npx pixels (one after another in y / out / da / dy; stat
 * [ng][2C]; work ng * fen_bn_work_floats(C)) in the same launches as one group -- each group its
 * own statistics, the running statistics and dgamma / dbeta moved group by group in order:
 * bit-identical to ng calls (the D step's real and fake batches, trainer.py:433-434).
 * fen_bn_apply_n takes group g's mean / rstd at mean / rstd + g * mstride.
 * A stride-2 conv = fen_conv3x3 at full resolution + fen_subsample2; its gradients = the
 * stride-1 ones of fen_zero_insert2(dy).                                                  */
size_t fen_bn_work_floats(int C);
int fen_bn_stats(int dtype, size_t npx, int C, const void* y, float eps, float momentum, float* stat, float* rmean,
                 float* rvar, float* work, void* stream);
int fen_bn_apply(int dtype, size_t npx, int C, const void* y, const float* mean, const float* rstd,
                 const float* gamma, const float* beta, float slope, void* out, void* stream);
int fen_bn_bwd(int dtype, size_t npx, int C, const void* da, const void* y, const float* stat, const float* gamma,
               const float* beta, float slope, void* dy, float* dgamma, float* dbeta, int accumulate, float* work,
               void* stream);
int fen_bn_stats_n(int dtype, int ng, size_t npx, int C, const void* y, float eps, float momentum, float* stat,
                   float* rmean, float* rvar, float* work, void* stream);
int fen_bn_apply_n(int dtype, int ng, size_t npx, int C, const void* y, const float* mean, const float* rstd,
                   int mstride, const float* gamma, const float* beta, float slope, void* out, void* stream);
int fen_bn_bwd_n(int dtype, int ng, size_t npx, int C, const void* da, const void* y, const float* stat,
                 const float* gamma, const float* beta, float slope, void* dy, float* dgamma, float* dbeta,
                 int accumulate, float* work, void* stream);
int fen_subsample2(int dtype, int B, int H, int W, int C, const void* x, void* y, void* stream);
/* space-to-depth by 2: y[b][i][j][(2a + c2) * C + c] = x[b][2i + a][2j + c2][c] (x [B,H,W,C] ->
 * y [B,H/2,W/2,4C]); inverse = 1 maps y back.  With the phase-major filter
 * W'[co][(2a + c2) C + c][kh'][kw'] = W[co][c][kh][kw] (kh = 1 -> a = 0, kh' = 1; kh = 0 ->
 * a = 1, kh' = 0; kh = 2 -> a = 1, kh' = 1; kw likewise) a stride-2 conv (discriminator.py:
 * 47-82) is a stride-1 conv of y at a quarter of the pixels, and its data gradient comes back
 * through the inverse.                                                                     */
int fen_s2d2(int dtype, int B, int H, int W, int C, const void* x, void* y, int inverse, void* stream);
/* that phase-major filter from W (gather = 0: W [Cout][C][3][3] fp32 -> W' [Cout][4C][3][3],
 * zeros where no tap lands) and the OIHW gradient back from the phase-major one (gather = 1)  */
int fen_s2d_filter(int Cout, int C, const float* src, float* dst, int gather, void* stream);
int fen_zero_insert2(int dtype, int B, int Ho, int Wo, int C, const void* dy, void* out, void* stream);

/* The discriminator's classifier head (discriminator.py:85-90, replaces its two nn.Linear and the
 * LeakyReLU between them; use_sigmoid 131-132), fp32: x [B][K] (the flattened NCHW features),
 * w1 [N][K], b1 [N], w2 [N] (= classifier.3.weight [1][N]), b2 [1].
 * fwd: pre [B][N] = x w1^T + b1 (kept for the backward), y [B] = LeakyReLU(pre, slope) w2 + b2
 *      (sigmoid = 1: its sigmoid).
 * bwd: gy [B] = dL/dy -> dx [B][K] (NULL: skipped), dw1 [N][K], db1 [N], dw2 [N], db2 [1], all
 *      written (not accumulated).
 * K a multiple of 256, N a multiple of 128 up to 1024 (else FEN_EUNSUPPORTED); work: fen_dhead_work_floats()
 * floats.  Fixed-order reductions: deterministic.                                             */
size_t fen_dhead_work_floats(int B, int K, int N);
int fen_dhead_fwd(int B, int K, int N, const float* x, const float* w1, const float* b1, const float* w2,
                  const float* b2, float slope, int sigmoid, float* pre, float* y, float* work, void* stream);
int fen_dhead_bwd(int B, int K, int N, const float* x, const float* w1, const float* pre, const float* w2,
                  const float* y, const float* gy, float slope, int sigmoid, float* dx, float* dw1, float* db1,
                  float* dw2, float* db2, float* work, void* stream);
/* GANLoss (discriminator.py:154-206) over n fp32 scores x against a constant label, mean
 * reduction: mode 0 'vanilla' nn.BCEWithLogitsLoss (torch's stable form), 1 'lsgan' nn.MSELoss,
 * 2 'wgan' target * x (target -1 for real, +1 for fake).  loss[0] = the mean; the gradient
 * gx = d(term)/dx / n * gy[0], gy the upstream gradient on the device.  FEN_EINVAL: mode, n.  */
int fen_gan_loss(int mode, int n, const float* x, float target, float* loss, void* stream);
int fen_gan_loss_bwd(int mode, int n, const float* x, float target, const float* gy, float* gx, void* stream);

/* A status word for fen_group_strip / fen_group_strip_bwd `status`: one zeroed int in
 * host-mapped, coherent pinned memory (hipHostMalloc, 64 B), allocated on the first call for
 * the current device and kept for the process; *host is what the host reads (no sync needed),
 * *dev what the kernels store to.  The only allocation the library makes.  0 or FEN_EHIP.  */
int fen_status_word(void** host, void** dev);
/* Read and clear a status word in one atomic exchange (a launch storing between a separate
 * read and clear would otherwise be lost); `host` is fen_status_word's *host.  Returns the
 * bits that were set (0: none).                                                            */
int fen_status_take(void* host);

/* Data-parallel gradient exchange (replaces DDP's bucketed all-reduce,
 * reference trainer.py:126-134 / scripts/train.py:325-330).  One communicator per process
 * (one process per GPU); each call of fen_rccl_allreduce_bucket is ONE in-place fp32 SUM
 * ncclAllReduce of a contiguous bucket of the flat gradient arena, enqueued on `stream` --
 * no host sync, no events, no watchdog, so it records into a hipGraph capture from any host
 * thread.  RCCL is resolved at run time (the instance already in the process, else
 * librccl.so.1).  The unique id (128 bytes) is made on one rank and distributed by the
 * caller (torch.distributed broadcast).  fen_rccl_init blocks until all nranks have joined
 * (ncclCommInitRank on `device`).  Errors: FEN_ERCCL + fen_last_rccl_error().              */
int fen_rccl_unique_id(void* id);
int fen_rccl_init(void** comm, const void* id, int nranks, int rank, int device);
int fen_rccl_allreduce_bucket(void* comm, float* buf, size_t count, void* stream);
int fen_rccl_check(void* comm);          /* ncclCommGetAsyncError: FEN_OK or FEN_ERCCL      */
int fen_rccl_destroy(void* comm);
const char* fen_last_rccl_error(void);
const char* fen_rccl_library(void);      /* which librccl was resolved ("none" if absent)   */

const char* fen_status_string(int code);
/* hipGetErrorString() of the HIP error behind this thread's last FEN_EHIP, or "none". */
const char* fen_last_hip_error(void);
const char* fen_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* FEN_H */
