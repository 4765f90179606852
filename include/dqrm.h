/*
 * dqrm.h — C ABI of libdqrm, the MI355X-native (gfx950 / CDNA4) implementation of
 * DQRM's data-parallel QAT step for embedding tables.
 *
 * Reference: YangZhou08/Deep_Quantized_Recommendation_Model_DQRM @ 2024-10-24.
 * Each entry point below names the reference interface it replaces (file:line).
 *
 * Conventions
 *  - Plain C: pointers, sizes, enums. No torch types. Every device pointer is a HIP
 *    device allocation owned by the caller; the library never allocates or frees
 *    caller memory and keeps no global device state.
 *  - Every call is stream-ordered on the hipStream_t passed as `void* stream`
 *    (NULL = the legacy default stream). No call synchronises the host except
 *    dqrm_read_errors().
 *  - Every call returns an int status: 0 = ok, <0 = error (see DQRM_E_*). The message
 *    of the last failing call on the calling thread is returned by dqrm_last_error().
 *    No C++ exception crosses the ABI.
 *  - Shapes: T tables, D = embedding dim (same for all tables, D % 4 == 0, D <= 256),
 *    B = bags per table per call, L_t = lookups of table t.
 *
 * Resident table state (one "table set" = all T tables of a model, one slab each):
 *    W        f32 [R][D]            FP32 master rows, table t = rows [row_base[t], +num_rows[t])
 *    packed   u8  [R][D/2]          INT4 rows, offset-binary nibbles (q+8), element 2j in the
 *                                   low nibble of byte j (FBGEMM/torch 4-bit rowwise order);
 *                                   nullable when the packed path is unused
 *    rowmax   f32 [R]               max_d |W[r][d]|
 *    blkmax   f32 [NB]              max of rowmax over 256-row blocks   (blk_base[t] per table)
 *    sblkmax  f32 [NS]              max of blkmax over 256-block (65536-row) superblocks
 *    tmax     f32 [T]               max of sblkmax over the table = max |W_t|
 *    scale    f32 [T]               embedding scale s_t used by the latest forward
 *    pscale   f32 [T]               scale the packed rows were built with (NaN = never)
 *    meta     i64 [4][T]            row_base, num_rows, blk_base, sblk_base (device copy)
 *
 *  The max hierarchy makes the reference's per-step full-table min/max
 *  (quant_utils.py:177-178, called every training forward at
 *  quant_modules_not_quantize_grad.py:337) exact and O(touched rows).
 */
#ifndef DQRM_H_
#define DQRM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQRM_ABI_VERSION 11 /* 2: dqrm_table_set.bdirty, dqrm_set_apply_kernel, dqrm_apply_local;
                               3: backward workspace (dqrm_bwd_workspace_bytes), no per-slot key cap;
                               4: dqrm_table_set.sync (in-launch hierarchy finalize), padded flags;
                               5: dqrm_emb_bwd_apply_local (coalesce + local update, one launch);
                               6: residency-checked one launch (dqrm_bwd_apply_local_is_one_launch),
                                  dqrm_checksum64 mixes the full 64-bit position,
                                  dqrm_table_set.num_rows_host;
                               7: dqrm_emb_fwd_after_update;
                               8: dqrm_comm (RCCL communicator owned by libdqrm), dqrm_exchange
                                  (the N > 1 exchange as two calls), dqrm_emb_bwd_lookup_grad_presum;
                               9: dqrm_emb_bwd_apply_fwd_local (the next batch's forward behind the
                                  one-launch update), dqrm_bwd_apply_fwd_local_is_one_launch,
                                  dqrm_emb_bwd_sgd_fwd;
                              10: dqrm_comm_init_external (a caller-served all-gather under the
                                  same exchange orchestration), dqrm_comm_size,
                                  dqrm_bwd_sgd_fwd_is_one_launch, DQRM_APPLY_MERGE,
                                  dqrm_apply_sparse_update_fwd, dqrm_apply_fwd_is_one_launch,
                                  dqrm_apply_workspace_bytes, dqrm_exchange.apply_ws,
                                  dqrm_exchange_apply_fwd;
                              11: the flat apply's finalize and the next forward in one launch
                                  (dqrm_apply_sparse_update_fwd), dqrm_apply_fwd_form */

/* status codes */
#define DQRM_OK            0
#define DQRM_E_INVALID    -1   /* bad argument (shape, null pointer, unsupported bits) */
#define DQRM_E_HIP        -2   /* HIP runtime error */
#define DQRM_E_CAPACITY   -3   /* a size exceeds this build's index range (e.g. max_lookups >= 2^30) */
#define DQRM_E_WORKSPACE  -4   /* workspace too small */

/* device-side error flags accumulated in dqrm_table_set.err (read with dqrm_read_errors) */
#define DQRM_ERRF_INDEX    1u  /* an index was outside [0, num_rows[t]) (reference: IndexError) */
#define DQRM_ERRF_OFFSET   2u  /* offsets not non-decreasing / outside [0, L_t] */
#define DQRM_ERRF_OVERFLOW 4u  /* a table had more lookups than dqrm_batch.max_lookups promised, or a
                                      caller-sized workspace / payload was too small */
#define DQRM_ERRF_STALL    8u  /* the workgroups of a fused launch could not all be resident at once
                                  (dqrm_emb_bwd_apply_local): its update is incomplete */

#define DQRM_BLOCK_ROWS   256     /* rows per blkmax entry */
#define DQRM_SBLOCK_ROWS  65536   /* rows per sblkmax entry */
#define DQRM_TABLE_SPLIT  8       /* workgroups (row-range slots) per table in the backward */
#define DQRM_SYNC_STRIDE  64      /* uint32 words between two tables' arrival counters */
#define DQRM_SLOT_KEYS    8192    /* merged payload entries the slot apply kernel sorts on chip
                                     (a fuller slot is applied by the flat method instead) */

/* Resident state of T tables. All pointers are device pointers. */
typedef struct dqrm_table_set {
    int32_t  num_tables;      /* T */
    int32_t  dim;             /* D */
    int64_t  total_rows;      /* R = sum num_rows */
    int64_t  total_blocks;    /* NB */
    int64_t  total_sblocks;   /* NS */
    float*   W;
    uint8_t* packed;          /* nullable */
    float*   rowmax;
    float*   blkmax;
    float*   sblkmax;
    float*   tmax;
    float*   scale;
    float*   pscale;
    const int64_t* meta;      /* [4][T]: row_base, num_rows, blk_base, sblk_base */
    uint32_t* err;            /* 1 word, device-side error flags */
    uint32_t* tflags;         /* [T] scratch (repack decision), library-internal */
    uint8_t*  sdirty;         /* [NS] zero-initialised scratch (superblock rescan flags); the
                                 allocation is readable up to the next 4-byte boundary */
    uint8_t*  bdirty;         /* [NB] zero-initialised scratch (block rescan flags), same padding */
    uint32_t* sync;           /* [T * DQRM_SYNC_STRIDE] zero-initialised scratch: per-table
                                 arrival counters of the updating kernels (the last workgroup
                                 of a table finalizes its |W| hierarchy inside the launch), one
                                 per 256 bytes; library-internal */
    const int64_t* num_rows_host; /* nullable HOST array [T]: the tables' row counts (meta's
                                 second row), for host-side launch planning (the one-launch local
                                 step gives its spare workgroups to the largest tables) */
} dqrm_table_set;

/* A batch of lookups for all T tables, in the reference's per-table
 * (lS_i[t], lS_o[t]) form (dlrm_data_pytorch.py:328-345, 1099-1157), concatenated:
 *   idx      i64 [sum_t L_t]  table t's indices at [idx_base[t], idx_base[t+1])
 *   off      i64 [T][B]       bag b of table t = idx_base[t] + [off[t][b], off[t][b+1])
 *                             (last bag ends at L_t), exactly nn.EmbeddingBag offsets
 *   idx_base i64 [T+1]        device copy
 * max_lookups must bound every L_t: it sizes the backward workspace (a table with more
 * lookups is skipped and flags DQRM_ERRF_OVERFLOW). There is no other per-batch limit. */
typedef struct dqrm_batch {
    const int64_t* idx;
    const int64_t* off;
    const int64_t* idx_base;
    int64_t  num_bags;        /* B */
    int64_t  max_lookups;     /* host upper bound on any L_t (capacity planning) */
    uint32_t flags;           /* DQRM_BATCH_* */
    uint32_t reserved;
} dqrm_batch;

/* Criteo form (dlrm_data_pytorch.py:328-345): every table has L_t == B (so idx_base[t] ==
 * t * B) and off[t][b] == b, i.e. bag b is lookup b. The kernels then read neither the
 * offsets nor idx_base. */
#define DQRM_BATCH_POOLING_ONE 1u

/* forward flags */
#define DQRM_FWD_REFRESH_SCALE 1u  /* s_t = clamp(tmax_t, 1e-8)/(2^(bits-1)-1), write scale[] */
#define DQRM_FWD_USE_PACKED    2u  /* single-lookup bags read INT4 rows (valid iff pscale==scale) */
#define DQRM_FWD_FULL_PRECISION 4u /* full_precision_flag: plain FP32 sum, no fake-quant */
#define DQRM_FWD_NT_STORE      16u /* stream the output with non-temporal stores (packed path) */

/* ---------------------------------------------------------------------------------
 * Table maintenance
 * ------------------------------------------------------------------------------ */

/* Full recompute of rowmax/blkmax/sblkmax/tmax from W (first forward, after
 * load_state_dict, after weight_syncc). Replaces the full-table scan of
 * quant_utils.py:141-194 (symmetric_linear_quantization_param_two). */
int dqrm_refresh_absmax(const dqrm_table_set* set, void* stream);

/* Periodic scale refresh + conditional repack (the stringified periodic-update path
 * quant_modules_not_quantize_grad.py:303-315,331-363). For each table:
 *   s_t = clamp(tmax_t, 1e-8) / (2^(bits-1)-1)   -> scale[t]
 *   if packed != NULL and pscale[t] != s_t: repack every row of t with s_t, pscale[t] = s_t.
 * Device-side decision; no host sync. bits must be 4 for repacking. */
int dqrm_refresh_scale_and_pack(const dqrm_table_set* set, int bits, void* stream);

/* ---------------------------------------------------------------------------------
 * Forward: fused multi-table INT4 fake-quant EmbeddingBag
 * Replaces QuantEmbeddingBagTwo.forward (quant_modules_not_quantize_grad.py:317-398)
 * called once per table by DLRM_Net.apply_emb (dlrm_s_pytorch_single_gpu.py:609-674):
 *   out = embedding_bag(idx, off, mode="sum")              (:367)
 *   q   = clamp(round(1/s * out + 0), -2^(b-1), 2^(b-1)-1)  (quant_utils.py:101,343)
 *   y   = q * s                                             (:393)
 * out[t][b][d] is written at out + t*out_stride_t + b*out_stride_b + d (floats).
 * Bags with one lookup may be served from the INT4 packed rows (bit-identical values
 * when pscale == scale); every other bag is summed in FP32 in bag order.
 * ------------------------------------------------------------------------------ */
int dqrm_emb_fwd(const dqrm_table_set* set, const dqrm_batch* batch, int bits,
                 uint32_t flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                 void* stream);

/* ---------------------------------------------------------------------------------
 * Backward workspace. The three backward calls below (SGD, coalesce, local update) sort
 * the lookups of every (table, row-range slot) by row on the device (in LDS up to 4096
 * lookups, in this workspace beyond) and process the distinct rows from a device-built
 * work list. Its size depends only on the table count and dqrm_batch.max_lookups: 16 bytes
 * up to 4096 lookups per table, T * DQRM_TABLE_SPLIT * max_lookups * 20 bytes beyond (each
 * of a table's row-range slots gets a spill region for all of the table's lookups, since a
 * slot's share is only known on the device; e.g. 26 tables x 1 M lookups = 4.2 GB).
 * Returns the bytes needed (0 on bad arguments). The workspace must be 16-B aligned; it
 * needs no initialisation (one call at a time per workspace).
 * ------------------------------------------------------------------------------ */
size_t dqrm_bwd_workspace_bytes(int num_tables, int64_t max_lookups);

/* ---------------------------------------------------------------------------------
 * Single-GPU backward + SGD, fused (no sparse gradient materialised).
 * Replaces: SymmetricQuantFunction.backward (quant_utils.py:349-363) + autograd of q*s,
 * EmbeddingBag sparse backward, and torch.optim.SGD.step on the sparse grad
 * (dlrm_s_pytorch_single_gpu.py:1736-1750,1943-1950). Per lookup i of row r, in lookup
 * order:  g' = (dy[bag(i)] * s) / s ;  W[r] = fma(g', -lr, W[r])   (torch CPU order).
 * ste = 0 skips the (g*s)/s step (forward ran with full_precision_flag).
 * Then rowmax/blkmax/sblkmax/tmax of touched rows, and (if packed != NULL and
 * repack_bits == 4) the touched INT4 rows with pscale.
 * ------------------------------------------------------------------------------ */
int dqrm_emb_bwd_sgd(const dqrm_table_set* set, const dqrm_batch* batch,
                     const float* dy, int64_t dy_stride_t, int64_t dy_stride_b,
                     int ste, float lr, int repack_bits, void* workspace, size_t workspace_bytes,
                     void* stream);

/* dqrm_emb_bwd_sgd on `batch`, then dqrm_emb_fwd(set, next, fwd_bits, fwd_flags, out, ...) on
 * the NEXT batch, with the same results as the two calls: the single-GPU driver's SGD step
 * (dlrm_s_pytorch_single_gpu.py:1943-1950) and the next apply_emb (:609-674), adjacent in its
 * loop. When the update takes the small-batch kernel (one workgroup per table, B <= 512
 * lookups) and `next` is a Criteo-form batch of the same size without DQRM_FWD_USE_PACKED,
 * each table's workgroup runs the next forward of that table itself right after its update:
 * one launch per step. Otherwise the two calls run. (A table whose batch overflows the
 * declared max_lookups is skipped and flagged, DQRM_ERRF_OVERFLOW, by the update and, in the
 * one-launch form, by its forward too.) */
int dqrm_emb_bwd_sgd_fwd(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                         int64_t dy_stride_t, int64_t dy_stride_b, int ste, float lr, int repack_bits,
                         void* workspace, size_t workspace_bytes, const dqrm_batch* next, int fwd_bits,
                         uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                         void* stream);

/* 1 if dqrm_emb_bwd_sgd_fwd would run the SGD of `batch` and the forward of `next` as ONE
 * launch (the small-batch kernel takes the update and `next` is a Criteo-form batch of the
 * same size without DQRM_FWD_USE_PACKED), 0 if as two launches, <0 on bad arguments. */
int dqrm_bwd_sgd_fwd_is_one_launch(const dqrm_table_set* set, const dqrm_batch* batch, const dqrm_batch* next,
                                   uint32_t fwd_flags);

/* ---------------------------------------------------------------------------------
 * Data-parallel gradient path (sgd_quantized_gradients_parallel_comm.py)
 *
 * Coalesced-gradient workspace (per rank). Slot k = t * DQRM_TABLE_SPLIT + s holds the
 * coalesced rows of table t that fall in row range s (ascending, unique):
 *   ws_cap_base i64 [T*S+1] (device)  slot k owns entries [ws_cap_base[k], ws_cap_base[k+1])
 *   ws_rows     i32 [WCAP]            local row ids
 *   ws_vals     f32 [WCAP][D]         coalesced sums
 *   ws_ucount   i32 [T*S]             entries used per slot
 *   ws_absmax   f32 [T*S]             partial maxima of |vals|: the max over table t's S
 *                                     entries is max |vals_t| (the local scale's input)
 * dqrm_coalesce_slot_caps() gives the slot capacities (host).
 * ------------------------------------------------------------------------------ */

/* Host helper: slot capacities cap[t*S+s] = min(max_lookups, rows in slot s of table t)
 * (a slot can never hold more distinct rows than that);
 * writes the exclusive prefix into ws_cap_base_host[T*S+1]; returns WCAP (>= 0). */
int64_t dqrm_coalesce_slot_caps(const int64_t* num_rows_host, int num_tables, int64_t max_lookups,
                                int64_t* ws_cap_base_host);

/* STE backward + EmbeddingBag sparse backward + grad.coalesce() (s_q_g_p_c.py:859),
 * plus the per-slot max |value| feeding the local scale
 * s_loc[t] = clamp(max|vals_t|, 1e-8) / (2^(bits-1)-1) (:861, quant_utils.py:141-194). */
int dqrm_emb_bwd_coalesce(const dqrm_table_set* set, const dqrm_batch* batch,
                          const float* dy, int64_t dy_stride_t, int64_t dy_stride_b,
                          int ste, const int64_t* ws_cap_base, int32_t* ws_rows, float* ws_vals,
                          int32_t* ws_ucount, float* ws_absmax, void* workspace, size_t workspace_bytes,
                          void* stream);

/* dqrm_emb_bwd_coalesce with every lookup's gradient divided by `divisor` before the
 * coalescing sum: values = sum over the row's lookups, in lookup order, of
 * ((dy*s)/s) / divisor -- the unquantized simulated-DP buffer of sgd_quantized_gradients.py:88-91
 * (embedding_grad_buffer.add_(grad / number_of_gpus); .coalesce()) when the batch holds the
 * N micro-steps' lookups back to back. Always the general (sorting) kernel; divisor 1 is
 * dqrm_emb_bwd_coalesce. */
int dqrm_emb_bwd_coalesce_scaled(const dqrm_table_set* set, const dqrm_batch* batch,
                                 const float* dy, int64_t dy_stride_t, int64_t dy_stride_b,
                                 int ste, int divisor, const int64_t* ws_cap_base, int32_t* ws_rows,
                                 float* ws_vals, int32_t* ws_ucount, float* ws_absmax, void* workspace,
                                 size_t workspace_bytes, void* stream);

/* Per-lookup (uncoalesced) sparse gradient, the COO nn.EmbeddingBag(mode="sum",
 * sparse=True) produces (embedding_bag_backward, sparse branch): for every lookup j of
 * table t, in lookup order, rows[j] = row_base[t] + idx[j] (slab row) and
 * vals[j][:] = (dy[t, bag(j)] * s_t) / s_t (ste != 0, quant_utils.py:349-363; s_t =
 * set->scale[t], the forward's scale) or dy[t, bag(j)]. j runs over the batch's flat
 * lookup positions (idx_base). The grad_mode="sparse" module hands this to
 * torch.optim.SGD (dlrm_s_pytorch_single_gpu.py:1943-1950), which then adds lookup by
 * lookup as with the reference's own embedding grad. rows i64 [L], vals f32 [L][D]. */
int dqrm_emb_bwd_lookup_grad(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                             int64_t dy_stride_t, int64_t dy_stride_b, int ste, int64_t* rows, float* vals,
                             void* stream);

/* Rows of W rewritten outside libdqrm -- torch.optim.SGD stepping on the
 * dqrm_emb_bwd_lookup_grad COO: recompute their row maxima, re-reduce their blocks,
 * superblocks and table maxima (the next refreshing forward's scale is then the full-table
 * max again, quant_utils.py:141-194) and, repack_bits == 4, repack their INT4 rows with the
 * frozen packing scale. rows: slab rows (device i64 [n], duplicates allowed). */
int dqrm_rows_changed(const dqrm_table_set* set, const int64_t* rows, int64_t n, int repack_bits, void* stream);

/* dqrm_rows_changed(set, rows, n, repack_bits) followed by dqrm_emb_fwd(set, batch, ...),
 * same results: the per-table module's sync after a torch.optim.SGD step on its COO grad
 * and its next forward (q_m_n_q_g.py:317-398 with the full-table scale of
 * quant_utils.py:141-194). A one-table set with a small batch (bags * D/4 <= 4096, n <= 4096,
 * FP32 rows, no repack) runs both as ONE single-workgroup launch; anything else as the two
 * calls. n == 0 is dqrm_emb_fwd. */
int dqrm_emb_fwd_after_update(const dqrm_table_set* set, const dqrm_batch* batch, int bits, uint32_t flags,
                              float* out, int64_t out_stride_t, int64_t out_stride_b, const int64_t* rows,
                              int64_t n, int repack_bits, void* stream);

/* Wire payload of one rank (bytes), produced by dqrm_grad_quant_pack:
 *   [counts i32 T*S | pad to 16] [rows i32 CAP | pad to 16] [vals CAP*D elems of
 *   int8 (bits<=8) / int16 (bits<=16) / f32 (bits==32, unquantized path)]
 * counts[t*S+s] = entries of table t in row-range slot s (S = DQRM_TABLE_SPLIT); table t's
 * entries sit at [cap_base[t], cap_base[t] + sum_s counts[t*S+s]), rows ascending, slot
 * after slot (so a receiving slot finds its entries without searching). */
size_t dqrm_payload_bytes(int num_tables, int64_t cap_total, int dim, int grad_bits);

/* Scale average + quantize-pack (s_q_g_p_c.py:861-869). absmax_all = the N ranks'
 * ws_absmax gathered [N][T*S]. Per table:
 *   s_r  = clamp(max_s absmax_all[r][t*S+s], 1e-8) / (2^(bits-1)-1)     (rank r's scale)
 *   s    = (((s_{N-1} + s_{N-2}) + ...) + s_0) * (1/N)
 *          (Gloo's one-element allreduce order; identical on every rank; -> s_avg)
 *   q    = clamp(round(1/s * v + 0), -2^(bits-1), 2^(bits-1)-1)  (quant_utils.py:101,343)
 * and the slots are compacted into the dense payload. grad_bits = 32 copies FP32 values
 * (emb_grad_quantized=False path, :319-327); absmax_all / s_avg may then be NULL. */
int dqrm_grad_quant_pack(int num_tables, int dim, const int64_t* ws_cap_base, int64_t ws_cap_total,
                         const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                         const float* absmax_all, int num_ranks, int grad_bits,
                         const int64_t* cap_base, int64_t cap_total, float* s_avg, void* payload,
                         void* stream);

/* dqrm_grad_quant_pack with the ranks' max|grad| rows absmax_pitch floats apart
 * (absmax_all[r * absmax_pitch + t*S + s]; >= T*S): one all-gather of several table sets'
 * concatenated ws_absmax serves every set (the DP hooks over a ModuleList of per-table
 * modules, sgd_quantized_gradients_parallel_comm.py). payload 16-B aligned. */
int dqrm_grad_quant_pack_strided(int num_tables, int dim, const int64_t* ws_cap_base, int64_t ws_cap_total,
                                 const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                                 const float* absmax_all, int64_t absmax_pitch, int num_ranks, int grad_bits,
                                 const int64_t* cap_base, int64_t cap_total, float* s_avg, void* payload,
                                 void* stream);

/* Ranking-range mixed-precision gradients (grad_precision_and_scale
 * s_q_g_p_c.py:158-255 decides a bit width per table: 0, 8 or 32). Quantize-pack with a
 * per-table bit width and scale (quantize_emb_grad_two, :836-848):
 *   table_bits[t] in 2..8 : q = clamp(round(1/table_scale[t] * v + 0), -2^(b-1), 2^(b-1)-1)
 *   table_bits[t] 0 or 32: the table sends no entries (grad_update_parallel_comm skips it, :280-289)
 * The payload layout is that of grad_bits = 8 (int8 values); apply it with
 * dqrm_apply_sparse_update(mode DQRM_UPD_DP, grad_bits 8, s_avg = table_scale). */
int dqrm_grad_quant_pack_ranked(int num_tables, int dim, const int64_t* ws_cap_base, int64_t ws_cap_total,
                                const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                                const int32_t* table_bits, const float* table_scale, const int64_t* cap_base,
                                int64_t cap_total, void* payload, void* stream);

/* Local (uncommunicated) update of the ranking-range 32-bit tables,
 * weight_update_parallel_comm :615-616  W.add_(-lr * grad)  with grad the rank's own sparse
 * gradient: per lookup, in lookup order, W[r] = W[r] + (g' * -lr) with g' = (dy*s)/s
 * (ste != 0), the product rounded separately. Only tables with table_mask[t] != 0
 * (NULL = all) are touched; rowmax/blkmax/sblkmax/tmax and (repack_bits == 4) packed rows
 * are maintained as in dqrm_emb_bwd_sgd. */
int dqrm_emb_local_update(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                          int64_t dy_stride_t, int64_t dy_stride_b, int ste, float lr, const int32_t* table_mask,
                          int repack_bits, void* workspace, size_t workspace_bytes, void* stream);

/* update modes for dqrm_apply_sparse_update */
#define DQRM_UPD_DP        0  /* v = ((Q * (1/N)) * s) ; W += -lr * v   (s_q_g_p_c.py:885,618-622) */
#define DQRM_UPD_SIMULATED 1  /* v = Q * f32((double)s / N) ; W += -lr * v (sgd_quantized_gradients.py:366-371) */
#define DQRM_UPD_FP32      2  /* v = (sum_r vals_r) * (1/N); W += -lr * v   (s_q_g_p_c.py:319-327,626) */

/* Decode N gathered payloads (contiguous, payload_bytes apart), union rows, integer
 * (or rank-ordered FP32) sum, dequantize and apply SGD to W; then maintain
 * rowmax/blkmax/sblkmax/tmax and (packed != NULL && repack_bits == 4) packed rows.
 * Replaces Gloo sparse all_reduce's coalesce (s_q_g_p_c.py:878) +
 * weight_update_parallel_comm (:601-628). */
int dqrm_apply_sparse_update(const dqrm_table_set* set, const int64_t* cap_base,
                             int64_t cap_total, const void* payloads, size_t payload_bytes,
                             int num_ranks, int grad_bits, const float* s_avg, float lr,
                             int mode, int repack_bits, void* stream);

/* dqrm_apply_sparse_update with rank r's payload at payloads + r * rank_pitch
 * (rank_pitch >= payload_bytes, multiple of 16): one all-gather of several sets'
 * concatenated payloads, each set decoding its own column of the gathered buffer. */
int dqrm_apply_sparse_update_strided(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total,
                                     const void* payloads, size_t payload_bytes, size_t rank_pitch, int num_ranks,
                                     int grad_bits, const float* s_avg, float lr, int mode, int repack_bits,
                                     void* stream);

/* dqrm_apply_sparse_update_strided on the gathered payloads, then dqrm_emb_fwd(set, next,
 * fwd_bits, fwd_flags, out, out_stride_t, out_stride_b) on the NEXT batch -- the same results as
 * those two calls (W, the |W| hierarchy, scale[] and out bit for bit). When the apply takes the
 * merge kernel (DQRM_APPLY_MERGE / AUTO at 1 < num_ranks <= 16) and `next` is a Criteo-form
 * batch without DQRM_FWD_USE_PACKED, the forward runs in the apply's launch: each table's
 * forward workgroups start once that table's update and |W| maxima are final (no finalize or
 * forward launch). When the flat apply kernel takes it (AUTO at num_ranks < dim/4) and the
 * forward reads the exact FP32 rows, the flat kernel's finalize and the forward share ONE launch
 * after it (the forward's index and row loads in flight while the table's maxima are finalized;
 * each table's scale taken once its finalize workgroup opened the table's gate). Reference: weight_update_parallel_comm (s_q_g_p_c.py:601-628) and the next
 * apply_emb (dlrm_s_pytorch_single_gpu.py:609-674, q_m_n_q_g.py:317-398). */
int dqrm_apply_sparse_update_fwd(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total,
                                 const void* payloads, size_t payload_bytes, size_t rank_pitch, int num_ranks,
                                 int grad_bits, const float* s_avg, float lr, int mode, int repack_bits,
                                 void* workspace, size_t workspace_bytes, const dqrm_batch* next, int fwd_bits,
                                 uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                                 void* stream);

/* Caller workspace of the merge apply at num_ranks > 1 (the positions of every entry's row in
 * every rank's payload: num_ranks^2 * cap_total ints; 0 at one rank). dqrm_apply_sparse_update_fwd
 * with a smaller workspace (or NULL) runs the flat apply kernel. next == NULL: the apply alone. */
size_t dqrm_apply_workspace_bytes(int num_ranks, int64_t cap_total);

/* 1 if dqrm_apply_sparse_update_fwd would run the update of num_ranks payloads (with that
 * workspace) and the forward of `next` with ONE update launch, 0 if not, <0 on bad arguments. */
int dqrm_apply_fwd_is_one_launch(const dqrm_table_set* set, int num_ranks, int64_t cap_total, size_t workspace_bytes,
                                 const dqrm_batch* next, uint32_t fwd_flags);

/* The launches dqrm_apply_sparse_update_fwd would issue for these arguments: DQRM_APPLY_FWD_SEPARATE
 * (the apply's launches, then the forward's), DQRM_APPLY_FWD_ONE_LAUNCH (update and forward in one
 * launch: the merge kernel) or DQRM_APPLY_FWD_FIN_FWD (the flat apply, then its finalize and the
 * forward in one launch); <0 on bad arguments. */
#define DQRM_APPLY_FWD_SEPARATE   0
#define DQRM_APPLY_FWD_ONE_LAUNCH 1
#define DQRM_APPLY_FWD_FIN_FWD    2
int dqrm_apply_fwd_form(const dqrm_table_set* set, int num_ranks, int64_t cap_total, size_t workspace_bytes,
                        const dqrm_batch* next, uint32_t fwd_flags);

/* Single-rank DP step (num_ranks == 1, mode DQRM_UPD_DP), dqrm_grad_quant_pack and
 * dqrm_apply_sparse_update fused: the table scale s = clamp(max_s ws_absmax[t*S+s], 1e-8)
 * / (2^(bits-1)-1) (-> s_avg[t]), q = quantize(v, s) per coalesced entry, and
 * W += -lr * ((q * 1) * s) straight from the coalesce workspace, with the same rounding
 * as the payload round trip (bit-identical W, rowmax/blkmax/sblkmax/tmax, s_avg and,
 * with repack_bits == 4, packed rows). No payload is written. Replaces, at world size 1,
 * quantize_emb_grad (s_q_g_p_c.py:861-869) + weight_update_parallel_comm (:601-628). */
int dqrm_apply_local(const dqrm_table_set* set, const int64_t* ws_cap_base, int64_t ws_cap_total,
                     const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                     const float* ws_absmax, int grad_bits, float* s_avg, float lr, int repack_bits,
                     void* stream);

/* World size 1: dqrm_emb_bwd_coalesce followed by dqrm_apply_local, with the same results
 * (W, the |W| hierarchy, s_avg, packed rows; the workspace's rows, counts and maxima -- its
 * values are scratch: a slot that fits keeps them on chip) -- for a
 * Criteo-form batch (DQRM_BATCH_POOLING_ONE, num_bags <= 4096, num_tables <= 32) in ONE
 * launch: each table's workgroups meet once to share their gradient maxima and then
 * update their row ranges, the W rows having been read during the coalesce. Replaces
 * quantize_emb_grad (s_q_g_p_c.py:850-869) + weight_update_parallel_comm (:601-628) at N=1,
 * the order grad_update_parallel_comm -> weight_update_parallel_comm runs them in
 * (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1895-1904). Other batches: the two calls.
 * The one launch needs its grid, (T+7)/8*64 workgroups of 1024 threads, resident at once:
 * it is taken only when the current device's CUs x the occupancy query cover the grid and
 * the stream's CU mask (hipExtStreamCreateWithCUMask) enables every CU; otherwise (a CPX
 * partition, a masked stream) the two calls run. A workgroup that still waits too long (other
 * streams' kernels holding CUs) does not update its rows and flags DQRM_ERRF_STALL: the update
 * of that step is then incomplete, never computed from a partial table maximum. */
int dqrm_emb_bwd_apply_local(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                             int64_t dy_stride_t, int64_t dy_stride_b, int ste, const int64_t* ws_cap_base,
                             int64_t ws_cap_total, int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount,
                             float* ws_absmax, int grad_bits, float* s_avg, float lr, int repack_bits,
                             void* workspace, size_t workspace_bytes, void* stream);

/* 1 if dqrm_emb_bwd_apply_local would run this batch as ONE launch on `stream` (the current
 * device), 0 if as the two calls, <0 on bad arguments. */
int dqrm_bwd_apply_local_is_one_launch(const dqrm_table_set* set, const dqrm_batch* batch, void* stream);

/* World size 1, the step boundary of a training loop: dqrm_emb_bwd_apply_local on `batch`,
 * then dqrm_emb_fwd(set, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b) on the
 * NEXT batch -- with the same results as those two calls (W and the |W| hierarchy, s_avg,
 * scale[] and out bit for bit). In the training loop these two are adjacent: the embedding
 * backward + update of step i (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1895-1904, at N=1)
 * and apply_emb of step i+1 (dlrm_s_pytorch_single_gpu.py:609-674, q_m_n_q_g.py:317-398),
 * whose indices the data loader has ready. When the update takes its one launch and `next`
 * is a Criteo-form batch of the same size without DQRM_FWD_USE_PACKED, the forward runs in
 * that launch: each table's workgroups, once the table's update and |W| maxima are final,
 * gather and fake-quantize the next batch's rows of that table (no second launch, no wait
 * for the other tables). Otherwise the two calls run. Error flags as the two calls'. */
int dqrm_emb_bwd_apply_fwd_local(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                                 int64_t dy_stride_t, int64_t dy_stride_b, int ste, const int64_t* ws_cap_base,
                                 int64_t ws_cap_total, int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount,
                                 float* ws_absmax, int grad_bits, float* s_avg, float lr, int repack_bits,
                                 void* workspace, size_t workspace_bytes, const dqrm_batch* next, int fwd_bits,
                                 uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                                 void* stream);

/* 1 if dqrm_emb_bwd_apply_fwd_local would run batch + next as ONE launch on `stream`, 0 if
 * not, <0 on bad arguments. */
int dqrm_bwd_apply_fwd_local_is_one_launch(const dqrm_table_set* set, const dqrm_batch* batch,
                                           const dqrm_batch* next, uint32_t fwd_flags, void* stream);

/* Which kernel dqrm_apply_sparse_update launches (process-wide; returns the previous
 * choice, or DQRM_E_INVALID). FLAT: one lane group per payload entry over the whole chip,
 * rows located in the other ranks' sorted row lists by binary search; SLOT: one workgroup
 * per (table, row-range slot), entries (row, rank) sorted in LDS. Both give bit-identical
 * results. AUTO (default; the environment variable DQRM_APPLY=flat|slot overrides it)
 * picks FLAT for num_ranks == 1 or num_ranks < dim/4 (one binary search per lane) and
 * SLOT above, where the per-entry searches cost more than the slot sort. */
#define DQRM_APPLY_AUTO 0
#define DQRM_APPLY_FLAT 1
#define DQRM_APPLY_SLOT 2
/* RANGES: one workgroup per block-aligned row range (a row-range slot cut in chunks) with
 * every rank's entries of it, rows owned: shrunk block maxima re-reduced in the workgroup,
 * the table's last workgroup re-reduces flagged superblocks -- no finalize launch
 * (DQRM_APPLY=ranges) */
#define DQRM_APPLY_RANGES 3
/* MERGE (opt-in, DQRM_APPLY=merge; <= 16 ranks, <= 64 tables; N > 1 needs the positions
 * workspace of dqrm_apply_sparse_update_fwd): k_merge_pos locates every entry's row in the other
 * ranks' payloads in LDS per block-aligned row range, k_apply_pos updates one lane group per entry
 * with the positions read in one load and finalizes the hierarchy in-launch; with a next batch its
 * forward runs in that launch behind per-table gates. Bit-exact with FLAT; not faster on the TB
 * shape, hence not AUTO. */
#define DQRM_APPLY_MERGE 4
int dqrm_set_apply_kernel(int kind);

/* Which backward kernels dqrm_emb_bwd_coalesce and dqrm_emb_bwd_sgd launch (process-wide;
 * returns the previous choice, or DQRM_E_INVALID). AUTO (default): batches in the Criteo
 * form (DQRM_BATCH_POOLING_ONE) with num_bags <= 4096 and max_lookups >= num_bags take the
 * Criteo-form coalesce kernel (dqrm_coalesce.hip), and SGD batches of at most 512 lookups
 * per table (fewer for D > 32) with num_bags * dim <= 16384 the one-workgroup-per-table SGD
 * kernel; everything else the general (sorting) kernel. GENERAL: always the general
 * kernel. Both give bit-identical results (coalesce: rows, values, counts, the max over a
 * table's DQRM_TABLE_SPLIT ws_absmax entries; SGD: W, the |W| maxima, packed rows). */
#define DQRM_COALESCE_AUTO 0
#define DQRM_COALESCE_GENERAL 1
int dqrm_set_coalesce_kernel(int kind);

/* ---------------------------------------------------------------------------------
 * Dense (MLP) layer gradients, data-parallel:
 *   quantize_linear_grad (per-channel) / quantize_bias_grad   s_q_g_p_c.py:892-961
 *   MLP branch of grad_update_parallel_comm                   s_q_g_p_c.py:337-409
 *   MLP branch of weight_update_parallel_comm                 s_q_g_p_c.py:630-668
 * A dense set is C "channels" over the bot_l/top_l Linear layers: every weight row is a
 * channel (per_channel=True, one scale per output feature) and every bias vector is one
 * channel (one scale per bias). Channel c is len[c] contiguous floats at grad[c] (the
 * layer's .grad) and param[c] (the layer's .data); its quantized values sit at
 * [wire_off[c], +len[c]) of the wire buffer. The arrays are device arrays.
 * Per step: scale -> all-gather of s_loc [C] -> quant -> all-reduce(SUM) of the wire ->
 * decode (grad_update_parallel_comm) ; update (weight_update_parallel_comm).
 * ------------------------------------------------------------------------------ */
typedef struct dqrm_dense_set {
    int32_t  num_channels;    /* C */
    int32_t  max_len;         /* max_c len[c] (host-side hint) */
    int64_t  total_elems;     /* wire elements = sum_c len[c] */
    float* const*  grad;      /* [C] device pointers to each channel's gradient */
    float* const*  param;     /* [C] device pointers to each channel's parameter */
    const int32_t* len;       /* [C] */
    const int64_t* wire_off;  /* [C] element offset of the channel in the wire */
} dqrm_dense_set;

/* wire element types of the quantized-gradient all-reduce */
#define DQRM_WIRE_F16 1  /* integer-valued fp16: exact sums for bits <= 8 and N <= 16 (|sum| <= 2048) */
#define DQRM_WIRE_I32 2  /* int32: exact for bits <= 16 */
#define DQRM_WIRE_F32 3  /* unquantized FP32 gradients (mlp_layer_quantized=False, :358-369) */

/* Host helper: the narrowest exact wire type for (bits, num_ranks); bits == 32 -> F32;
 * <0 if unsupported. */
int dqrm_dense_wire_type(int bits, int num_ranks);

/* Local per-channel scale (:905-912, quant_utils.py:196-220):
 *   s_loc[c] = clamp(max(|min_j g|, |max_j g|), 1e-8) / (2^(bits-1)-1). */
int dqrm_dense_grad_scale(const dqrm_dense_set* set, int bits, float* s_loc, void* stream);

/* Scale average + quantize into the wire (:913-918 / :945-950). s_all = the N ranks'
 * s_loc gathered [N][C]:
 *   s_avg[c] = (((s_{N-1} + s_{N-2}) + ...) + s_0) * (1/N)   (same order on every rank)
 *   wire     = clamp(round(1/s_avg[c] * g + 0), -2^(bits-1), 2^(bits-1)-1)
 * wire_type F32 copies the gradient unquantized (s_all, s_avg unused, may be NULL). */
int dqrm_dense_grad_quant(const dqrm_dense_set* set, int bits, const float* s_all, int num_ranks,
                          float* s_avg, int wire_type, void* wire, void* stream);

/* After the wire's all-reduce(SUM): grad = 0 + wire * (1/N)  (:920-922 then the hook's
 * grad.zero_(); grad.add_(buffer_changes), :345-351). */
int dqrm_dense_grad_decode(const dqrm_dense_set* set, const void* wire, int wire_type, int num_ranks,
                           void* stream);

/* weight_update_parallel_comm, MLP branch (:641-642 / :659-660):
 *   param += (-lr * grad) * s[c]     (s == NULL: param += -lr * grad, :644-645). */
int dqrm_dense_update(const dqrm_dense_set* set, const float* s, float lr, void* stream);

/* ---------------------------------------------------------------------------------
 * Row-wise PTQ formats of the reference's inference path.
 * DLRM_Net.quantize_embedding (dlrm_s_pytorch_single_gpu_documentingp.py:689-704) packs
 * each trained table with torch.ops.quantized.embedding_bag_{4bit,byte}_prepack and
 * apply_emb (:648-663) gathers with embedding_bag_{4bit,byte}_rowwise_offsets (mode sum,
 * optional per-sample weights). Byte-identical to those ops (FBGEMM fused row-wise):
 *   bits 4: row = D/2 bytes (element 2j low nibble, 2j+1 high) | fp16 scale | fp16 bias
 *   bits 8: row = D bytes | f32 scale | f32 bias
 * dim must be 8, 16, 32, 64, 128 or 256. W is 16-byte aligned, packed 4-byte aligned.
 * ------------------------------------------------------------------------------ */
/* Bytes per packed row (0 if bits/dim unsupported). */
size_t dqrm_rowwise_row_bytes(int bits, int dim);

/* packed[num_rows * row_bytes] <- prepack(W[num_rows, dim] f32).
 * Replaces torch.ops.quantized.embedding_bag_4bit_prepack / embedding_bag_byte_prepack. */
int dqrm_rowwise_prepack(int bits, const float* W, int64_t num_rows, int dim, uint8_t* packed,
                         void* stream);

/* out[num_bags, dim] f32 <- sum over bag b of dequant(packed[idx[i]]) (* per_sample_weights[i]),
 * accumulated in bag order as acc = fma(scale*w, q, acc + bias*w) (FBGEMM EmbeddingSpMDM).
 * Bag b covers idx[off[b] .. off[b+1]); with include_last_offset == 0 the last bag ends at
 * num_lookups, otherwise off has num_bags+1 entries. per_sample_weights may be NULL. Out-of-range indices are
 * skipped and flag DQRM_ERRF_INDEX in *err, bad offsets flag DQRM_ERRF_OFFSET (device
 * word, cleared by the caller). Replaces torch.ops.quantized.embedding_bag_4bit_rowwise_offsets /
 * embedding_bag_byte_rowwise_offsets (mode=0 sum). */
int dqrm_rowwise_bag(int bits, const uint8_t* packed, int64_t num_rows, int dim, const int64_t* idx,
                     int64_t num_lookups, const int64_t* off, int64_t num_bags, int include_last_offset,
                     const float* per_sample_weights, float* out, uint32_t* err, void* stream);

/* ---------------------------------------------------------------------------------
 * Criteo input path
 * One record = 40 int32: label, 13 dense, 26 categorical (the flat binary file that
 * data_loader_terabyte.numpy_to_binary writes, :243-280). dqrm_criteo_unpack replaces
 * CriteoBinDataset.__getitem__'s _transform_features (data_loader_terabyte.py:68-87,
 * :227-237) and the Kaggle collate (dlrm_data_pytorch.py:328-345) on a device-resident
 * record block records[num_samples][40]:
 *   dense  f32 [B][13]  = log(float(x_int) + 1)
 *   lS_i   i64 [26][B]  = x_cat (% max_ind_range if > 0, Python remainder), transposed
 *   labels f32 [B]      = float(label)
 *   lS_o   i64 [26][B]  = b (nullable: DQRM_BATCH_POOLING_ONE makes it unnecessary)
 * dense's log is the device logf (<= 2 ulp from torch's CPU log; integers bit-exact).
 * ------------------------------------------------------------------------------ */
#define DQRM_CRITEO_RECORD_INTS 40
#define DQRM_CRITEO_DENSE       13
#define DQRM_CRITEO_SPARSE      26

int dqrm_criteo_unpack(const int32_t* records, int64_t num_samples, int32_t max_ind_range, float* dense,
                       int64_t* lS_i, float* labels, int64_t* lS_o, void* stream);

/* ---------------------------------------------------------------------------------
 * Misc
 * ------------------------------------------------------------------------------ */
/* Synthetic on-device init U(-sqrt(1/n_t), +sqrt(1/n_t)) from a counter-based hash
 * (same distribution as quant_modules_not_quantize_grad.py:273-275; not numpy's stream). */
int dqrm_init_uniform(const dqrm_table_set* set, uint64_t seed, void* stream);

/* ---------------------------------------------------------------------------------
 * Replica synchronisation: weight_syncc (sgd_quantized_gradients_parallel_comm.py:963-970,
 * all_reduce(param, SUM) then param *= 1/N, every 200 iterations of the DP driver,
 * dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1801,1924-1936).
 * ------------------------------------------------------------------------------ */
/* *out (device u64, caller-zeroed) += sum_i mix64(word_i ^ i * 0xD1B54A32D192ED03) over num_words 32-bit
 * words of data (16-B aligned): a position-dependent, order-free 64-bit checksum whose
 * all-gather tells whether every rank holds the same bits. */
int dqrm_checksum64(const void* data, int64_t num_words, uint64_t* out, void* stream);

/* In place, the reference's all-reduce + scale of num_replicas IDENTICAL replicas of data:
 * x = fl(fl(...fl(x + x) + x ...) * inv_n), num_replicas - 1 sequential adds -- the order in
 * which a ring all-reduce (Gloo ring_chunked, RCCL ring) accumulates the ranks. Bit-exact
 * with that all-reduce when every rank holds x; the identity for num_replicas 1, 2 and 4
 * with inv_n = 1/num_replicas (barring overflow of num_replicas * x), not for 3 or 8. */
int dqrm_replica_mean(float* data, int64_t n, int num_replicas, float inv_n, void* stream);

/* ---------------------------------------------------------------------------------
 * The N > 1 exchange over RCCL (xGMI), issued from the library: the reference's 52 blocking
 * Gloo collectives per step (2 per table, sgd_quantized_gradients_parallel_comm.py:865,878)
 * become two ncclAllGather calls per step on a communicator libdqrm owns, each stream-ordered
 * between the step's kernels, with no host round trip in between.
 * ------------------------------------------------------------------------------ */
typedef struct dqrm_comm dqrm_comm;

/* RCCL's unique id (128 bytes) for dqrm_comm_init; called by one rank, which hands it to
 * the others (the Python layer broadcasts it over the torch.distributed process group). The
 * RCCL library is the one already loaded in the process (PyTorch's), else librccl.so.1. */
int dqrm_comm_unique_id(void* id128);

/* Collective over the `nranks` processes (one per GPU, each with the same id): creates this
 * rank's communicator on the current HIP device. nranks == 1 is allowed (local copies). */
int dqrm_comm_init(dqrm_comm** comm, int nranks, int rank, const void* id128);

/* A communicator whose all-gather the caller serves: every dqrm_comm_allgather on it (and so
 * both collectives of dqrm_exchange_grad) calls fn(send, recv, bytes, stream, user) on the
 * issuing host thread, with the device pointers and the stream the call was given, in the
 * step's order. fn must leave recv[r * bytes, (r+1) * bytes) = rank r's send in stream order
 * before the stream's next work (e.g. a torch.distributed all_gather_into_tensor on that
 * stream, or a Gloo gather staged through host memory after a stream synchronise) and return
 * 0, else non-zero (the exchange call then fails with DQRM_E_HIP). The exchange's kernels and
 * buffer handling are those of the RCCL communicator: this is how the N > 1 orchestration runs
 * over the reference's own transport (Gloo, s_q_g_p_c.py:865,878) or torch.distributed's. */
typedef int (*dqrm_allgather_fn)(const void* send, void* recv, size_t bytes, void* stream, void* user);
int dqrm_comm_init_external(dqrm_comm** comm, int nranks, int rank, dqrm_allgather_fn fn, void* user);
int dqrm_comm_destroy(dqrm_comm* comm);
int dqrm_comm_size(const dqrm_comm* comm);

/* recv[r * bytes, (r+1) * bytes) <- rank r's send[0, bytes), in rank order, on `stream`
 * (ncclAllGather of bytes uint8). */
int dqrm_comm_allgather(dqrm_comm* comm, const void* send, void* recv, size_t bytes, void* stream);

/* One rank's exchange state, all device buffers caller-owned and reused every step (the
 * Python SparseGradExchange builds it once). */
typedef struct dqrm_exchange {
    const dqrm_table_set* set;
    dqrm_comm* comm;            /* NULL: world size 1, no collective (num_ranks must be 1) */
    int32_t num_ranks;          /* the communicator's size */
    int32_t grad_bits;          /* 2..16 quantized, 32 = the unquantized FP32 path */
    const int64_t* ws_cap_base; /* the coalesced-gradient workspace (dqrm_emb_bwd_coalesce) */
    int64_t ws_cap_total;
    int32_t* ws_rows;
    float* ws_vals;
    int32_t* ws_ucount;
    float* ws_absmax;           /* [T*S] this rank's per-slot max|grad| */
    float* absmax_all;          /* [num_ranks][T*S] gathered maxima (world size 1 without comm: ws_absmax) */
    const int64_t* cap_base;    /* [T+1] payload capacity prefix */
    int64_t cap_total;
    float* s_avg;               /* [T] the averaged gradient scale (emb_scaling_factor) */
    void* payload;              /* this rank's wire payload, dqrm_payload_bytes */
    void* gathered;             /* [num_ranks][payload_bytes] (world size 1 without comm: payload) */
    size_t payload_bytes;
    void* workspace;            /* backward scratch, dqrm_bwd_workspace_bytes(T, max_lookups) */
    size_t workspace_bytes;
    void* apply_ws;             /* the merge apply's positions, dqrm_apply_workspace_bytes(num_ranks,
                                   cap_total); NULL / too small: the flat apply kernel */
    size_t apply_ws_bytes;
} dqrm_exchange;

/* grad_update_parallel_comm's embedding branch for all tables (s_q_g_p_c.py:257-317 via
 * quantize_emb_grad :850-890) in one call: dqrm_emb_bwd_coalesce -> all-gather of the per-slot
 * maxima -> dqrm_grad_quant_pack_strided (rank scales averaged in Gloo's order) -> all-gather
 * of the payloads. Same results as those calls made one by one. */
int dqrm_exchange_grad(const dqrm_exchange* x, const dqrm_batch* batch, const float* dy,
                       int64_t dy_stride_t, int64_t dy_stride_b, int ste, void* stream);

/* weight_update_parallel_comm's embedding branch (s_q_g_p_c.py:601-628): decode the gathered
 * payloads and apply (dqrm_apply_sparse_update_strided with mode / repack_bits). */
int dqrm_exchange_apply(const dqrm_exchange* x, float lr, int mode, int repack_bits, void* stream);

/* dqrm_exchange_apply followed by the NEXT batch's forward, dqrm_emb_fwd(x->set, next, fwd_bits,
 * fwd_flags, out, out_stride_t, out_stride_b): dqrm_apply_sparse_update_fwd on the gathered
 * payloads -- the update of step i and apply_emb of step i+1, adjacent in the DP loop
 * (dlrm_s_pytorch_tb_dp_one_parallel_comm.py:1888-1904, then the next iteration's forward). */
int dqrm_exchange_apply_fwd(const dqrm_exchange* x, float lr, int mode, int repack_bits, const dqrm_batch* next,
                            int fwd_bits, uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                            void* stream);

/* dqrm_emb_bwd_lookup_grad with duplicate rows pre-summed: same rows[], but vals[j] is the
 * sum, in lookup order, of the STE'd dy rows of every lookup of row idx[j] when j is the
 * row's FIRST lookup, and +0.0 for its later lookups. Handed to torch.optim.SGD
 * (dlrm_s_pytorch_single_gpu.py:1943-1950) the scatter-add then adds one value per row
 * (a zero entry adds -lr * 0 = -0.0, the identity), so W is bit-identical run to run;
 * the COO sums to the same per-row gradient. Tables of more than DQRM_PRESUM_MAX_LOOKUPS
 * lookups: DQRM_E_CAPACITY (nothing written). */
#define DQRM_PRESUM_MAX_LOOKUPS 2048
int dqrm_emb_bwd_lookup_grad_presum(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                                    int64_t dy_stride_t, int64_t dy_stride_b, int ste, int64_t* rows,
                                    float* vals, void* stream);

/* Synchronises `stream`, returns the accumulated DQRM_ERRF_* flags in *flags and
 * clears them (if clear != 0). */
int dqrm_read_errors(const dqrm_table_set* set, uint32_t* flags, int clear, void* stream);

const char* dqrm_last_error(void);
int dqrm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DQRM_H_ */
