/* Diagnostic entry points of libmignn.so (timing studies only, not product
 * ABI).  See gnn-bfs-rans_amd/csrc/diag.hip. */
#ifndef MIGNN_DIAG_H
#define MIGNN_DIAG_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* Ablation / schedule flags of the fused layer kernels, OR-ed with the
 * MIGNN_EPI_* flags; accepted only by the mignn_diag_* entry points below
 * (the product entry points of mignn.h reject them): results are wrong by
 * design for the NO_* ablations. */
enum {
    MIGNN_DIAG_NO_PRODUCE = 256,      /* skip the A-tile producer */
    MIGNN_DIAG_NO_MFMA = 512,         /* skip the MFMA + store */
    MIGNN_SCHED_XCD_MAJOR = 1024,     /* exact-fp32 tile kernel: XCD-major tile order */
    MIGNN_DIAG_TRACE = 2048,          /* s_memtime timeline (mignn_diag_set_trace*) */
    MIGNN_DIAG_NO_EXT = 4096,         /* f16x3 GCN layer: skip the out-of-tile gathers */
    MIGNN_DIAG_NO_LOCAL = 8192,       /* f16x3 GCN layer: skip the in-tile (LDS) pass */
    MIGNN_DIAG_NO_TABLES = 16384,     /* f16x3 GCN layer: skip the lookup-table build */
    MIGNN_DIAG_PLAIN_STORE = 32768,   /* split-fp16 GEMM: unstaged (16 x 64-B) row stores */
    MIGNN_SCHED_INTERLEAVED = 65536,  /* f16x3 GCN layer: step s covers tiles [sG, (s+1)G) (the
                                         default: each XCD walks a contiguous tile range) */
    MIGNN_SCHED_PRIO_CONSUMERS = 131072, /* f16x3 GCN layer: consumer waves at s_setprio 1 */
    MIGNN_SCHED_PRIO_PRODUCERS = 262144, /* f16x3 GCN layer: producer waves at s_setprio 1 */
    MIGNN_SCHED_DMA_LATE = 524288,       /* f16x3 GCN layer: own-row DMA after the epilogue */
    MIGNN_SCHED_NC8 = 1048576            /* f16x3 GCN layer: 8 consumer waves (16 columns each) */
};
/* mignn_gcn_layer / mignn_gcn_layer_f16x3 / mignn_linear with the flags above */
int mignn_diag_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* ew,
                         const float* x, int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                         const float* w, const float* bias, const float* scale,
                         const float* shift, int flags, float* out, int64_t ldo, void* stream);
int mignn_diag_gcn_layer_f16x3(const int32_t* row_ptr, const int32_t* col, const float* ew,
                               const float* x, int64_t ldx, int64_t row_begin, int64_t row_end,
                               int h, const float* w, const float* bias, const float* scale,
                               const float* shift, int flags, float* out, int64_t ldo,
                               void* stream);
int mignn_diag_linear(const float* a, int64_t lda, int64_t m, int k, const float* a2,
                      int64_t lda2, int k2, const float* w, int n, const float* bias,
                      const float* residual, int64_t ldr, const float* scale, const float* shift,
                      int flags, float* c, int64_t ldc, void* stream);
/* mignn_linear_f16x3 with MIGNN_DIAG_NO_PRODUCE (no A loads), NO_MFMA (no
 * MFMAs), NO_EXT (no C stores) */
int mignn_diag_linear_f16x3(const float* a, int64_t lda, int64_t m, int k1, const float* a2,
                            int64_t lda2, int k2, const void* img, int n, const float* bias,
                            const float* residual, int64_t ldr, const float* scale,
                            const float* shift, int flags, float* c, int64_t ldc, void* stream);

/* mode 0: CSR gather (h = 128); 1: stencil gather on the periodic grid;
 * 3: copy in the 16x16 MFMA-tile store pattern (16 rows x 64 B per instruction);
 * 2: streaming copy.  blocks <= 0: one row group per row. */
int mignn_diag_gather(int mode, const int32_t* row_ptr, const int32_t* col, const float* ew,
                      const float* x, int64_t n, int nx, int ny, int nz, int blocks, float* out,
                      void* stream);
/* Timeline buffer (uint64 [8 * 64 * 8], device memory) for launches with
 * MIGNN_DIAG_TRACE: s_memtime stamps per workgroup 0..7 and step 0..63 --
 * slot 0/1 producer step start / gather done, 2/3/4 consumer step start /
 * MFMA done / epilogue done.  NULL disables. */
int mignn_diag_set_trace(void* buf);
/* The same for mignn_gcn_layer_f16x3 (uint64 [8 * 64 * 4]): slot 0/1 producer
 * wave 0 step start / aggregation done, 2/3 consumer wave 0 after the
 * residual hand-off / before the step's barrier. */
int mignn_diag_set_trace_f16x3(void* buf);

/* Fused output head (H = 128, out_dim 7) timing ablations: mode 4 = MFMA
 * segments at raised wave priority (exact results); mode bit 1 = no x
 * loads, bit 2 = no MFMAs (results wrong by design). */
/* Shader clock probe: `blocks` workgroups of 4*iters dependent FMAs each;
 * out[2b] = s_memtime delta, out[2b+1] = s_memrealtime delta (100 MHz). */
/* v_pk_fma_f32 forms of the row-code expansion (0 scalar chain, 1 inline
 * asm with op_sel_hi:[1,0,1], 2 inline asm without it, 3 compiler-packed);
 * codes [n, 8], coef [h, 8], out [n, h] */
int mignn_diag_pk_fma(int form, const float* codes, int64_t n, const float* coef, int h,
                      float* out, void* stream);
int mignn_diag_clock(int blocks, int iters, int64_t* out, void* stream);

int mignn_diag_mlp_head(int mode, const float* x, int64_t n, const void* img, float* out,
                        void* stream);

/* Fused H = 256 layers (csrc/agg_gemm.hip) timing ablations, OR-ed into every
 * launch until reset with 0 (results wrong by design): NO_PRODUCE = no
 * aggregate sums, NO_MFMA = no MFMAs, NO_EXT = no out-of-tile row DMA,
 * NO_TABLES = no own-row chunk DMA, NO_LOCAL = no epilogue, SCHED_INTERLEAVED =
 * no W chunk DMA. */
int mignn_diag_set_fused_flags(int flags);
/* mignn_gat_layer: 1 (default) = the fused kernel where it applies, 0 = the
 * aggregate + transform launches (timing study) */
int mignn_diag_set_gat_fused(int on);
#ifdef __cplusplus
}
#endif
#endif
