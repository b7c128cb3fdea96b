/*
 * spai_hip.h — C ABI of libspai_hip.so, the MI355X (gfx950) hot path of SPAI-via-GFlowNet.
 *
 * The reference (tonylizza/gflownet-spai @ 2024-10-24) is pure Python/PyTorch with no
 * FFI; its hot path is the call chain
 *     GFlowNet.sample_states  (gflownet/gflownet.py:125-197)
 *       -> ForwardPolicy logits + Categorical sampling (policy.py:34-73, gflownet.py:148)
 *       -> PreconditionerEnv.update (preconditioner.py:32-52)
 *            -> update_edges_and_convert_to_sparse + resize (gflownet/utils.py:295-356, 89-126)
 *            -> calculate_residual ||M A - I||_F (preconditioner.py:79-93)
 *            -> evaluate_preconditioner / reward (preconditioner.py:55-66, 137-165)
 * Each entry point below names the reference code it replaces.  The Python drop-ins
 * (gflownet_spai_amd/{gflownet,preconditioner,log}.py) bind these through ctypes; the
 * binding a maintainer would add to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer owned by the caller, unless noted.
 *     No allocation crosses the ABI; the library uses only the caller's workspace.
 *   - `stream` is a hipStream_t passed as void*; all calls are stream-ordered and
 *     asynchronous (no host synchronisation inside any call).
 *   - Return value: SPAI_OK (0) or an error code; spai_last_error() returns a
 *     thread-local message for the last failing call.  Nothing throws across the ABI.
 *   - Bitmaps are uint32 words, bit (a & 31) of word (a >> 5) <=> action / edge a.
 *   - "Lines" are the ELL rows of a sparse matrix in one orientation: for the
 *     ||M A - I|| side (reference) line i = row i (CSR), for the ||A M - I|| side
 *     (north star) line j = column j (CSC).  A pattern line holds, per slot, the other
 *     index (-1 = padding), the action id of that entry and its initial value.
 */
#ifndef SPAI_HIP_H
#define SPAI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPAI_OK 0
#define SPAI_ERR_INVALID 1     /* bad argument (maps to ValueError) */
#define SPAI_ERR_HIP 2         /* HIP runtime / launch failure (RuntimeError) */
#define SPAI_ERR_UNSUPPORTED 3 /* shape outside the compiled kernels (NotImplementedError) */

#define SPAI_FILL_COPY 0 /* M = pattern values of kept entries (gflownet/utils.py:331-353) */
#define SPAI_FILL_LSQ 1  /* m_j = argmin ||A[:,J_j] m - e_j||_2 (north-star extension) */

#define SPAI_DTYPE_F32 0
#define SPAI_DTYPE_F64 1

/* ABI version (bumped on any signature change) and last error text. */
int spai_abi_version(void);
const char* spai_last_error(void);

/* ---------------------------------------------------------------- per-launch kernel timing
 * HIP-event durations of single kernels inside the multi-kernel entry points, measured on the
 * launch stream (bench.py's roofline objects need the kernel's own average duration, not its
 * phase's).  spai_kernel_timer_arm(kernel, 1) clears the kernel's records and arms it: every
 * later launch of that kernel records a start / stop event pair on its stream (at most 256 pairs;
 * none while the stream is being captured into a graph); arm(kernel, 0) stops recording.
 * spai_kernel_timer_read waits for the recorded events and returns their count and mean duration
 * in ms.  Process-wide, not re-entrant.  kernel: */
#define SPAI_TIMER_TILE 0  /* k_tile of spai_rollout_select(_pm): the step's dominant kernel */
#define SPAI_TIMER_SORT 1  /* k_sort2 of spai_rollout_sort */
#define SPAI_TIMER_QR 2    /* k_qr_solve of spai_fill_lines_qr_cached (the bench's fill) */
#define SPAI_TIMER_GRAM 3  /* k_gram_fill / k_gram_fill_wide of spai_fill_lines_gram(_dict) */
#define SPAI_TIMER_COUNT 4
int spai_kernel_timer_arm(int32_t kernel, int32_t on);
int spai_kernel_timer_read(int32_t kernel, int32_t* count, double* avg_ms);

/* ---------------------------------------------------------------- logits statistics
 * lmax[b] = max_a logits[b, a], z[b] = sum_a exp(logits[b, a] - lmax[b]) (fp64), over the
 * E1 = E + 1 actions of each of B rows spaced `bstride` floats apart (bstride 0 = one row
 * shared by all samples; outputs are still written for every b).
 * Replaces the softmax normaliser of policy.py:73 (computed once per rollout because
 * the reference's logits are state-independent within a rollout, gflownet.py:133,145). */
size_t spai_logits_stats_workspace_bytes(int32_t E1, int32_t B);
int spai_logits_stats(const float* logits, int64_t bstride, int32_t E1, int32_t B,
                      float* lmax, double* z, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- reference-parity step
 * One step of the reference loop (gflownet.py:135-179): for every sample b,
 *   a_b = argmax_a w_a / noise[b, a],  w_a = exp(l_a - lmax_b), w_a := 0 if chosen,
 * i.e. Categorical(probs).sample() == argmax(p / q), q ~ Exp(1) (torch multinomial
 * fast path; noise drawn on the host from the torch CPU generator, B*(E+1) per step).
 * For active samples: sets the chosen bit, logs out_action[b] = a_b and
 * out_prob[b] = w_a / zrem[b] (log.py:70), subtracts w_a from zrem[b] and clears
 * active[b] when a_b == E (gflownet.py:177-179).  Inactive samples log -1 and 1.0.
 * chosen: [B][words1] bitmap over E+1 actions. */
size_t spai_parity_step_workspace_bytes(int32_t E1, int32_t B);
int spai_parity_step(const float* logits, int64_t bstride, int32_t E1, int32_t B, const float* noise,
                     const float* lmax, uint32_t* chosen, int32_t words1, uint8_t* active, double* zrem,
                     int64_t* out_action, float* out_prob, void* workspace, size_t workspace_bytes,
                     void* stream);

/* ---------------------------------------------------------------- throughput rollout
 * Whole trajectories in one pass (replaces the T-step loop of gflownet.py:135-179) as an
 * exponential race: action a arrives at t_a = q_a * r_a, q_a = -ln u_a (u from Philox4x32-10
 * with counter (a >> 2, sample_base + b, stream_lo, stream_hi) and key (seed_lo, seed_hi)),
 * r_a = e^(l_E - l_a) (r_E = 1); the removed set of sample b is {a < E : t_a < t_E} and the
 * trajectory lists it by t ascending (ties: action ascending), i.e. the Gumbel keys
 * l_a - ln q_a in descending order.  Distributionally identical to the reference's sequential
 * sampling without replacement; bit-exact to oracle/ (arrival_times, throughput_rollout).
 *
 * Phase 1 (spai_rollout_select): writes removed[B][words] (words = ceil(E/32)), stages the
 * winners in the workspace grouped by presampled time buckets, and (nparts = 1) counts[B]
 * (= k_b, the number removed).
 * Phase 2 (spai_rollout_sort, then spai_rollout_finish; spai_rollout_order = both): sorts
 * each bucket in LDS and writes the trajectory log in [B][t_cap] layout (t_cap >= E + 1, only
 * the first T columns are written, T = max_b k_b + 1 is stored to *t_out):
 *   actions[b][t] = t-th removed action, actions[b][k_b] = E, -1 up to T;
 *   fwd_probs[b][t] = w_{a_t} / (W_rest + sum_{s>=t} w_{a_s}), w = exp(l - lmax), W_rest =
 *   mass of the actions never removed (terminal included) = the masked-softmax probability
 *   of step t (policy.py:65-73, log.py:70), 1.0 after the terminal;
 * (log.py:67-87 semantics: the Log's actions [T,B] is the transpose).  lmax comes from
 * spai_logits_stats (or the policy's k_max).  One workspace serves both phases of one rollout;
 * phase 2 may be repeated on the same select (it is idempotent).
 *
 * stream_ctr (optional, device uint64): when non-null the Philox stream id is read from it
 * instead of `stream_id`, and the select phase adds 1 to it (a captured HIP graph of the
 * rollout then draws a fresh rollout on every replay).
 *
 * Parts (the multi-GPU split): the presampled splitters cut every sample's
 * winners into nb buckets in trajectory order; part p of nparts owns buckets
 * [nb*p/nparts, nb*(p+1)/nparts), i.e. one contiguous slice of every trajectory.  Every part
 * draws all E actions (removed and the untouched mass are complete on every part), but only
 * its own winners are bucketed, staged and sorted.  Its select fills the exchange array
 * (spai_rollout_ws_offset fields 2/6: per-bucket weight sums and winner counts of its own
 * buckets, 0 elsewhere, then B * SPAI_RES2_LIMBS caller slots); the caller sums that array over
 * the parts (an all-reduce of its int64 bit patterns: every entry is non-zero on one part only,
 * so the sum equals the one-part array bit for bit, and the slots carry the exact residual
 * limbs), then calls
 * spai_rollout_merge (counts, T, bucket positions and masses), spai_rollout_sort (actions and
 * fwd_probs of its slice) and spai_rollout_finish (the last part writes the terminal step and
 * the padding; t_out is written by every part). */
size_t spai_rollout_workspace_bytes(int32_t E, int32_t B);
/* Persistent grid of the sort phase (spai_rollout_sort's k_sort2, one whole CU per block): at most
 * `blocks` blocks (0 = one per CU, the default), so a kernel launched on another stream beside the
 * sort (the fill) keeps the remaining CUs.  Process-wide setting. */
int spai_set_sort_blocks(int32_t blocks);
int spai_rollout_select(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                        uint64_t seed, uint64_t stream_id, uint64_t* stream_ctr, int32_t sample_base,
                        int32_t part, int32_t nparts, uint32_t* removed, int32_t words, int32_t* counts,
                        void* workspace, size_t workspace_bytes, void* stream);
/* spai_rollout_select with the logits maximum still to be formed (the small launches):
 * lmax_parts [n_lmax_parts] = the block maxima spai_policy_logits left with B = 0; one extra block
 * of the select's first launch reduces them and writes lmax[0..B-1] (an output here) before its
 * first reader.  One shared logits row only (bstride 0).  Otherwise identical to
 * spai_rollout_select (same outputs, bits and workspace). */
int spai_rollout_select_pm(const float* logits, int64_t bstride, int32_t E, int32_t B, float* lmax,
                           const float* lmax_parts, int32_t n_lmax_parts, uint64_t seed, uint64_t stream_id,
                           uint64_t* stream_ctr, int32_t sample_base, int32_t part, int32_t nparts,
                           uint32_t* removed, int32_t words, int32_t* counts, void* workspace,
                           size_t workspace_bytes, void* stream);
int spai_rollout_merge(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                       int32_t part, int32_t nparts, int32_t* counts, void* workspace, size_t workspace_bytes,
                       void* stream);
int spai_rollout_sort(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                      int32_t part, int32_t nparts, int64_t t_cap, int64_t* actions, float* fwd_probs,
                      void* workspace, size_t workspace_bytes, void* stream);
int spai_rollout_finish(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                        const int32_t* counts, int32_t part, int32_t nparts, int64_t t_cap, int64_t* actions,
                        float* fwd_probs, int32_t* t_out, void* workspace, size_t workspace_bytes, void* stream);
int spai_rollout_order(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                       const int32_t* counts, int64_t t_cap, int64_t* actions, float* fwd_probs,
                       int32_t* t_out, void* workspace, size_t workspace_bytes, void* stream);
/* Byte offset inside the rollout workspace (tests, the multi-part exchange): field 0 = int32
 * oversized buckets the last sort handed to the global-memory sort, 1 = int32 T of the last
 * rollout, 2 = fp64 exchange array ([B][2][kMaxB] bucket weight sums | bucket winner counts,
 * then [B][SPAI_RES2_LIMBS] int64 caller slots), 4 = int32 [B][kMaxB + 1] trajectory position of each bucket's first
 * winner, 5 = int32 [B] buckets per sample (a part's slice of sample b is
 * [pos[b][nb*p/np], pos[b][nb*(p+1)/np])); field 3 returns kMaxB itself, field 6 the length of
 * the exchange array in fp64 values.  -1 for an unknown field or bad shape. */
int64_t spai_rollout_ws_offset(int32_t E, int32_t B, int32_t field);

/* ---------------------------------------------------------------- generic residual
 * res2_out[b] = sum over lines l in [line_begin, line_end) of
 *   || sum_p M_b[l][p] A_line(idx_b[l][p]) - e_l ||^2
 * for B ARBITRARY sparse M_b given as ELL lines (rows: ||M A - I||_F^2, columns: ||A M - I||_F^2;
 * replaces the sparse torch.mm + identity subtraction + torch.norm of preconditioner.py:79-93,
 * the calculate_residual of any M): m_idx [B][n][W] int32 (-1 = empty slot, sample stride
 * idx_bstride elements, 0 = one index set for every sample), m_val [B][n][W] (stride
 * val_bstride), A lines [n][WA].  Widths W <= 5/7/13 with WA <= 5/7; fp64 accumulation.
 * Workspace: spai_residual_workspace_bytes(line_end - line_begin, B). */
size_t spai_residual_workspace_bytes(int32_t n_lines, int32_t B);
int spai_residual_lines(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, const int32_t* m_idx,
                        int64_t idx_bstride, const void* m_val, int32_t m_dtype, int64_t val_bstride, int32_t WA,
                        const int32_t* a_idx, const void* a_val, int32_t a_dtype, int32_t B, double* res2_out,
                        void* workspace, size_t workspace_bytes, void* stream);
/* The same sums with the index matching taken from a pattern's Gram cache (lines of M 5 / 7 / 13
 * wide over A lines <= 5 / 7 / 7 wide, A values fp32 or fp32-exact narrowed): pat_idx [n][W] the pattern's
 * indices, gram_dict / line_entry its Gram cache as a dictionary (spai_gram_build's blocked
 * cache -> spai_line_cache_dict: distinct entries of W(W+1)/2 + W values, gram_dtype fp32/fp64;
 * 16-byte aligned).
 * A line of sample b whose every slot holds the pattern's index or -1 (the candidates of the
 * fixed pattern) reads its G, c from the cache; any other line is matched from A as above.
 * The result is bit-identical to spai_residual_lines when the cache is the pattern's over this A
 * (the caller's contract: it is not checked). SPAI_ERR_UNSUPPORTED for other widths / dtypes. */
int spai_residual_lines_gram(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, const int32_t* m_idx,
                             int64_t idx_bstride, const void* m_val, int32_t m_dtype, int64_t val_bstride, int32_t WA,
                             const int32_t* a_idx, const void* a_val, int32_t a_dtype, const int32_t* pat_idx,
                             const void* gram_dict, int32_t gram_dtype, const int32_t* line_entry, int32_t B,
                             double* res2_out, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- actions -> removal sets
 * removed[b] = { a : 0 <= a < E, a in actions[b, :] } (preconditioner.py:37-43 +
 * utils.py:315-323: -1 padding and the terminal id E are ignored), and
 * counts[b] = |removed[b]|, so nnz(M_b) = E - counts[b] (utils.py:343-353 coalesce). */
int spai_actions_to_removed(const int64_t* actions, int64_t stride_b, int64_t stride_t, int32_t B,
                            int32_t T, int32_t E, uint32_t* removed, int32_t words, int32_t* counts,
                            void* stream);

/* ---------------------------------------------------------------- exact residual sums
 * The squared residual of a batch is a sum of per-block fp64 partials.  Each partial is
 * truncated toward zero to a multiple of 2^-96 and summed as integers: SPAI_RES2_LIMBS int64
 * slots per sample (six signed 32-bit limbs, value = sum_i L_i 2^(32 i - 96), then a count of
 * non-representable partials: NaN in bits 32.., inf or |x| >= 2^94 in bits 0..31, then a pad).
 * Integer addition is associative, so the slots of a sample summed over ANY partition of its
 * lines into 256-line-aligned ranges (the column shards of a multi-GPU job: one all-reduce SUM
 * of the int64 slots) give the same bits as one launch over all lines; res2 = the slots'
 * value rounded once to fp64 (NaN / +inf when flagged). */
#define SPAI_RES2_LIMBS 8
int spai_res2_from_limbs(int32_t B, const int64_t* limbs, double* res2_out, void* stream);

/* ---------------------------------------------------------------- fill + residual
 * For lines [line_begin, line_end) of the pattern and every sample b:
 *   keep_p = (pat_idx[l,p] >= 0) && !removed[b][pat_act[l,p]]
 *   fill_mode COPY: m_p = keep_p ? (float)pat_val[l,p] : 0        (utils.py:331-353)
 *   fill_mode LSQ : m = argmin ||A_lines[J] m - e_l||, J = kept p  (north star; fp64 solve)
 *   res2_out[b]  = sum over the lines of || sum_p m_p A_line(pat_idx[l,p]) - e_l ||^2 (fp64)
 * which is ||M A - I||_F^2 (row lines, CSR; preconditioner.py:79-93) or ||A M - I||_F^2
 * (column lines, CSC) restricted to those lines; summing res2_out over a partition of
 * the lines (e.g. the ranks of a column-sharded job) gives the full square norm.
 * M is evaluated from its STORED precision (m_dtype).  m_out (may be NULL) receives
 * [B][line_end - line_begin][W] values in m_dtype (0 where not kept).
 * Bitmap windows: row b of `removed` (row stride `words` uint32) holds bitmap words
 * word_base, word_base + 1, ... of sample b (word_base 0, words = ceil(E/32): whole bitmaps);
 * every word an action id of the lines names must lie inside the row (a column shard needs
 * only the words its lines' action ids span: the multi-GPU all-to-all ships just those).
 * res2_out (fp64 [B]) and/or limbs_out ([B][SPAI_RES2_LIMBS], the exact sums above) receive
 * the per-sample sums; either may be NULL, not both.
 * a_idx/a_val: [n][WA] lines of the original matrix A (n x n) in the same orientation.
 * Widths W, WA <= 7 run the register kernel (one thread per line, all samples); wider
 * COPY lines run the LDS hash kernel (one workgroup per line, every sample; A lines read up to
 * their first -1 slot, i.e. left-packed ELL; up to 13000 distinct entries in a line of the
 * product, a line with more gets a NaN residual); anything else returns SPAI_ERR_UNSUPPORTED. */
size_t spai_fill_workspace_bytes(int32_t n_lines, int32_t B);
int spai_fill_residual(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                       const int32_t* pat_idx, const int32_t* pat_act, const float* pat_val, int32_t WA,
                       const int32_t* a_idx, const void* a_val, int32_t a_dtype, int32_t B,
                       const uint32_t* removed, int32_t words, int32_t word_base, void* m_out, int32_t m_dtype,
                       double* res2_out, int64_t* limbs_out, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- Gram-cached fill + residual
 * The LSQ fill and the residual of line l need only G_pq = <A_line(k_p), A_line(k_q)> and
 * c_p = A_line(k_p)[l] over the line's pattern slots p (other index k_p); both depend on the
 * pattern and A only, and the candidate pattern is fixed per PreconditionerEnv
 * (preconditioner.py:23-25).  spai_gram_build computes them once per env for all n lines
 * into `gram` (spai_gram_bytes(n, W) bytes, fp64, blocked [ceil(n/64)][T + Wc][64] with
 * Wc = 5 (W <= 5), 7 (W <= 7) or 13 (W <= 13; A widths WA <= 7), T = Wc(Wc+1)/2: the
 * packed upper triangle of G, then c).
 * spai_fill_residual_gram then does what spai_fill_residual does (same fill modes,
 * res2_out / m_out semantics, line range, precision rules) from pat_act (+ pat_val for
 * COPY) and `gram` alone: per-rollout traffic is a stream of the line data and, per sample,
 * the mask bits and M values.  Widths above 13 (or WA above 7) return SPAI_ERR_UNSUPPORTED
 * (use spai_fill_residual; its LSQ mode covers W <= 7).  Workspace: spai_fill_workspace_bytes(line_end - line_begin, B).
 * spai_gram_compact writes the same entries as fp32 (same blocked layout, half the bytes) and
 * clears *exact (caller sets it to 1) if any entry changes in the fp64 -> fp32 -> fp64 round
 * trip; only an exact copy may be used (gram_dtype SPAI_DTYPE_F32, widths W <= 13): the fill
 * then computes bit for bit what it computes from the fp64 cache (e.g. integer stencils,
 * whose G and c are small integers), with 80 instead of 160 bytes per 5-wide line. */
size_t spai_gram_bytes(int32_t n, int32_t W);
int spai_gram_build(int32_t n, int32_t W, const int32_t* pat_idx, int32_t WA, const int32_t* a_idx,
                    const void* a_val, int32_t a_dtype, double* gram, void* stream);
int spai_gram_compact(int32_t n, int32_t W, const double* gram, float* gram32, int32_t* exact, void* stream);
int spai_fill_residual_gram(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                            const int32_t* pat_act, const float* pat_val, const void* gram, int32_t gram_dtype,
                            int32_t B, const uint32_t* removed, int32_t words, int32_t word_base, void* m_out,
                            int32_t m_dtype, double* res2_out, void* workspace, size_t workspace_bytes,
                            void* stream);
/* The two halves of spai_fill_residual_gram: the fill kernel leaves per-block (256-line) fp64
 * partial sums in the workspace; spai_fill_reduce (n_lines = line_end - line_begin of that
 * call) sums them per sample exactly (SPAI_RES2_LIMBS) into res2_out and/or limbs_out. */
int spai_fill_lines_gram(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                         const int32_t* pat_act, const float* pat_val, const void* gram, int32_t gram_dtype, int32_t B,
                         const uint32_t* removed, int32_t words, int32_t word_base, void* m_out, int32_t m_dtype,
                         void* workspace, size_t workspace_bytes, void* stream);
int spai_fill_reduce(int32_t n_lines, int32_t B, const void* workspace, double* res2_out, int64_t* limbs_out,
                     void* stream);
/* One GPU (the lines are all of M): spai_fill_reduce + spai_rewards in one launch, from the
 * workspace spai_fill_lines_gram left (n_lines = all n lines); same outputs as spai_rewards. */
int spai_fill_reduce_rewards(int32_t n_lines, int32_t B, const void* workspace, const int32_t* removed_counts,
                             int64_t nnz0, int32_t n, double r0, double f0, const float* alpha, double* residual,
                             double* reward, float* reward32, void* stream);

/* ---------------------------------------------------------------- least squares by Householder QR
 * The LSQ fill of spai_fill_residual (m = argmin ||A_lines[J] m - e_l||, J = the kept slots of line
 * l) solved by Householder QR of the line's dense block instead of the normal equations: per line
 * the rows I the slots' A lines touch are merged (ascending) into D = A[I, slots] in LDS, and every
 * sample's masked problem is factored on a group of lanes (reflection norms and dot products by DPP
 * lane swaps); a slot is dropped when its remaining column norm is below 1e-12 of its full norm
 * (fp64 rank deficiency; the normal-equations fill drops below 1e-13 of the SQUARED norm, i.e.
 * ~3e-7 of the norm, so it loses nearly dependent columns the QR fill still resolves).  The line
 * residual^2 is ||Q^T e_l||^2 below the pivots
 * (+1 when l is not in I).  Same outputs and workspace as spai_fill_lines_gram: m_out (may be NULL)
 * [B][line_end - line_begin][W] in m_dtype, per-block partials for spai_fill_reduce /
 * spai_fill_reduce_rewards.  Pattern lines need pat_idx (other index) and pat_act; A lines a_idx /
 * a_val [n][WA] (a_dtype F32 when every value is exact in fp32: the same numbers, staged in half
 * the LDS).  Widths W <= 13 with WA <= 7 (W <= 5 needs WA <= 5, W <= 7 needs WA <= 7).
 * max_rows: spai_qr_max_rows' result for this pattern and A (the largest |I|; it selects the group
 * size: up to 16 / 32 / 64 / 96 rows); a line with more rows than the instance holds yields a NaN
 * residual.  No reference counterpart (the reference copies the pattern values, utils.py:331-353). */
int spai_qr_max_rows(int32_t n, int32_t W, const int32_t* pat_idx, int32_t WA, const int32_t* a_idx,
                     int32_t* max_rows, void* stream);
int spai_fill_lines_qr(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, const int32_t* pat_idx,
                       const int32_t* pat_act, int32_t WA, const int32_t* a_idx, const void* a_val, int32_t a_dtype,
                       int32_t max_rows, int32_t B, const uint32_t* removed, int32_t words, int32_t word_base,
                       void* m_out, int32_t m_dtype, void* workspace, size_t workspace_bytes, void* stream);
/* The same fill split at its sample-independent boundary.  The per-line Householder QR of the
 * full block D = A[I, slots] depends on A and the pattern only, both fixed for an env's lifetime
 * (preconditioner.py:23-25), so it runs ONCE per env (spai_qr_factor) into an R cache: per line the
 * packed R (W(W+1)/2), Q^T e_l (W) and the tail ||(Q^T e_l)[W..]||^2 (+1 when l is not in I), fp64,
 * blocks of 64 lines structure-of-arrays (spai_qr_cache_bytes; W = the width class 5 / 7 / 13 of
 * (W, WA) as spai_fill_lines_qr).  Per rollout, spai_fill_lines_qr_cached reads the cache and the
 * pattern's action ids, one thread per line: the kept columns R_J re-triangularised by Householder
 * reflections of at most W rows (R_J has the singular values of A[I, J]: no normal equations),
 * back-substitution, the same rank floor (the column norms are recomputed as sum_i R_ip^2) and the
 * same outputs / workspace / partial layout as spai_fill_lines_qr (width classes 5, 7 and 13; the
 * 13-wide class re-reads its line's R per sample).  No reference counterpart (utils.py:331-353 copies). */
size_t spai_qr_cache_bytes(int32_t n, int32_t W, int32_t WA);
int spai_qr_factor(int32_t n, int32_t W, const int32_t* pat_idx, const int32_t* pat_act, int32_t WA,
                   const int32_t* a_idx, const void* a_val, int32_t a_dtype, int32_t max_rows, double* rcache,
                   size_t rcache_bytes, void* stream);
/* line_entry: NULL, or rcache is the cache's dictionary (spai_line_cache_dict) of `entries` entries
 * and line_entry [n] names each line's entry.  With a dictionary of <= 4096 entries and the 5-wide
 * class, every (entry, keep mask) solution is computed once per call into an (entry, mask) table
 * placed in the workspace after the partials (at the first 256-byte boundary past
 * ceil((line_end - line_begin) / 256) * B doubles; entries * 32 * 6 doubles; without that room the
 * per-line solves run) and each (line, sample) reads its M values and residual from it: the same
 * arithmetic on the same values, so the same bits as solving it on the line's own lane (ABI 19). */
int spai_fill_lines_qr_cached(int32_t n, int32_t line_begin, int32_t line_end, int32_t W, int32_t WA,
                              const int32_t* pat_act, const double* rcache, const int32_t* line_entry,
                              int32_t entries, int32_t B, const uint32_t* removed, int32_t words, int32_t word_base,
                              void* m_out, int32_t m_dtype, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- cache dictionaries
 * The dictionary of a per-line cache in the blocked layout of spai_qr_factor / spai_gram_build
 * (value q of line j at ((j / 64) * nq + q) * 64 + j % 64, elem_bytes 8 or 4): its distinct line
 * entries, compared bitwise, into dict ([entries][nq] contiguous) and per line the index of its
 * entry into line_entry [n].  *entries_out = the number of distinct entries, or max_entries + 1
 * (nothing written) when there are more.  Env setup: synchronises `stream` and reads the cache
 * back to the host.  A stencil's interior lines share one entry (the same A values in the same
 * relative positions give the same R / Gram values bit for bit), so the per-rollout fills
 * (spai_fill_lines_qr_cached with line_entry, spai_fill_lines_gram_dict) read 4 bytes per line
 * instead of nq values and run the same arithmetic on the same values: the same bits.  The wide
 * (8-13) Gram fill re-reads its dictionary entry per sample instead of holding it in registers
 * (two waves per SIMD instead of one).  No reference counterpart (env-constant layout). */
int spai_line_cache_dict(int32_t n, int32_t nq, int32_t elem_bytes, const void* cache, size_t cache_bytes,
                         int32_t max_entries, void* dict, size_t dict_bytes, int32_t* line_entry,
                         int32_t* entries_out, void* stream);
int spai_fill_lines_gram_dict(int32_t fill_mode, int32_t n, int32_t line_begin, int32_t line_end, int32_t W,
                              const int32_t* pat_act, const float* pat_val, const void* dict, int32_t gram_dtype,
                              const int32_t* line_entry, int32_t B, const uint32_t* removed, int32_t words,
                              int32_t word_base, void* m_out, int32_t m_dtype, void* workspace,
                              size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- multi-GPU bitmap exchange
 * The columns split's all_to_all send buffer (gflownet_spai_amd/distributed.py; the reference has
 * no parallelism, its per-sample loop is preconditioner.py:37-51).  For destination q < P and
 * candidate b < bl: the removal bits removed[b] (row stride `words`) of the action ids
 * ids[seg[q] .. seg[q+1]) — q's line-major action ids — packed 32 per word (bit j of the segment
 * -> word j / 32, bit j % 32), then counts[b].  q's block starts at out + out_off[q] and is
 * [bl][wq + 1] words, wq = ceil((seg[q+1] - seg[q]) / 32).  max_seg = the longest segment.  The
 * receiver reads the packed rows through shard-local action ids (0 .. seg length - 1 in the same
 * line-major order), so every rank receives nnz(shard) bits per candidate for ANY numbering of
 * the matrix (raw COO order defines the action ids, preconditioner.py:23-25). */
int spai_bitmap_pack(int32_t P, int32_t bl, const uint32_t* removed, int32_t words, const int32_t* counts,
                     const int32_t* ids, const int64_t* seg, const int64_t* out_off, int64_t max_seg, uint32_t* out,
                     void* stream);
/* The same send buffer for a numbering whose shards' action ids lie in compact bitmap windows
 * (a stencil in row-major raw order: rank q's ids span its rows +- the stencil's reach, about 1/P
 * of the bitmap), without the gather (ABI 20): q's block at out + out_off[q] is [bl][span[q] + 1]
 * words = removed[b][lo[q] .. lo[q] + span[q]) (row stride `words`), then counts[b].  The
 * receiver reads bit (a - 32 lo[rank]) of its rows for action id a.  lo, span, out_off: [P] int64
 * in device memory; max_span = max span[q] <= words.  distributed.PackPlan picks this layout when
 * the windows total <= 1.25x the packed words. */
int spai_window_pack(int32_t P, int32_t bl, const uint32_t* removed, int32_t words, const int32_t* counts,
                     const int64_t* lo, const int64_t* span, const int64_t* out_off, int64_t max_span, uint32_t* out,
                     void* stream);

/* ---------------------------------------------------------------- forward policy
 * logits[a] = fc(mean_pool(relu(GATv2_2(relu(GATv2_1(x))))))[a] for a < num_actions and
 * lmax[0..B-1] = max_a logits[a]: ForwardPolicy.forward up to the masked softmax
 * (policy.py:34-73, BasePolicy policy.py:14-21; GATv2Conv heads 4 then 1, edge_dim 1,
 * negative slope 0.2, concat, bias), evaluated once per rollout because the state graph
 * of gflownet.py:223-257 does not change within a rollout (gflownet.py:133,145).
 *   x       [n_nodes][fin] node features (state_to_data: ones(2N, 1))
 *   rowptr/src/eattr  the graph as a CSR by TARGET (edge_index[1]) over n_nodes, with self
 *           loops removed and one loop per node re-added whose attribute is the mean of the
 *           node's incoming attributes (GATv2Conv add_self_loops fill_value="mean")
 *   gat1/gat2  packed fp32 parameters of each layer: W_l [HC][F], b_l [HC], W_r [HC][F],
 *           b_r [HC], W_e [HC], att [HC], bias [HC]  (layer 1: F = fin, HC = 4 hid;
 *           layer 2: F = 4 hid, HC = hid); spai_policy_params(layer, fin, hid) floats each
 *   fc_w    [num_actions][hid] row-major (nn.Linear weight rows, 16-byte aligned), fc_b [num_actions]
 *   const_rows  non-zero when every row of x equals row 0 (spai_policy_rows_constant; the
 *           reference's x = ones(2N, 1) is): both GATv2 layers then give every node
 *           relu(W_l x0 + b_l + bias) (the attention weights of a target sum to 1), so the
 *           stack collapses to two small products and only the fc GEMV runs (rowptr, src,
 *           eattr may be null).  0: the general GATv2 kernels.
 * Compiled for fin in {1, 2, 4} and hid in {4, 8, 16, 32} (else SPAI_ERR_UNSUPPORTED).
 * Workspace: spai_policy_workspace_bytes(n_nodes, hid, num_actions). */
size_t spai_policy_params(int32_t layer, int32_t fin, int32_t hid);
/* B = 0 in spai_policy_logits defers the maximum: lmax then receives the fc kernel's per-block
 * maxima (spai_policy_lmax_parts(num_actions) floats) and no reduction launch runs; the rollout's
 * spai_rollout_select_pm reduces them (one launch fewer per step). */
int32_t spai_policy_lmax_parts(int32_t num_actions);
size_t spai_policy_workspace_bytes(int32_t n_nodes, int32_t hid, int32_t num_actions);
/* *flag = 1 if every row of x [n_nodes][fin] equals row 0, else 0 (asynchronous, on stream). */
int spai_policy_rows_constant(int32_t n_nodes, int32_t fin, const float* x, int32_t* flag, void* stream);
int spai_policy_logits(int32_t n_nodes, int32_t fin, int32_t hid, const float* x, const int32_t* rowptr,
                       const int32_t* src, const float* eattr, const float* gat1, const float* gat2,
                       const float* fc_w, const float* fc_b, int32_t num_actions, float* logits, float* lmax,
                       int32_t B, int32_t const_rows, void* workspace, size_t workspace_bytes, void* stream);
/* Backward of the same network (the TB loss's path into ForwardPolicy's parameters, autograd
 * through policy.py:34-73): given dlogits [num_actions], the gradients in the parameter packs'
 * layouts (g_gat1 / g_gat2: spai_policy_params floats each) and of the fc rows < num_actions
 * (g_fc_w [num_actions][hid], g_fc_b [num_actions]).  The forward is recomputed inside.
 * rev_ptr [n+1] / rev_eid [n_edges]: the CSR's edges grouped by source node (edge positions),
 * n_edges = rowptr[n] (self loops included).  hid 4 or 8, fin 1/2/4 (else SPAI_ERR_UNSUPPORTED).
 * Deterministic (fixed-order fp64 sums).  Workspace: spai_policy_backward_workspace_bytes. */
size_t spai_policy_backward_workspace_bytes(int32_t n_nodes, int32_t n_edges, int32_t fin, int32_t hid,
                                            int32_t num_actions);
int spai_policy_backward(int32_t n_nodes, int32_t n_edges, int32_t fin, int32_t hid, const float* x,
                         const int32_t* rowptr, const int32_t* src, const float* eattr, const int32_t* rev_ptr,
                         const int32_t* rev_eid, const float* gat1, const float* gat2, const float* fc_w,
                         int32_t num_actions, const float* dlogits, float* g_gat1, float* g_gat2, float* g_fc_w,
                         float* g_fc_b, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- training
 * Gradient of the logged forward probabilities w.r.t. the logits (the backward of
 * log.py:70 fwd_probs through policy.py:65-73's masked softmax, as trajectory_balance_loss
 * gflownet/utils.py:228-278 differentiates it):
 *   grad[a] (+)= sum_b sum_t gprobs[b,t] * d probs[b,t] / d logits[a]
 * with probs[b,t] = w_{a_t} / (untouched mass + sum_{s>=t} w_{a_s}), w = exp(logits - lmax[b]).
 *   logits   [E+1] (bstride 0: shared by all samples, grad_out [E+1] summed over b) or
 *            [B][bstride] (grad_out [B][E+1])
 *   actions  [B][lda] int64, the first T columns: removed actions, then E, then -1
 *   probs    [B][ldp] the rollout's fwd_probs; gprobs [B][ldg] = dL/dprobs
 *   removed  [B][words] the rollout's removal bitmaps (untouched = bit clear, a < E)
 * Deterministic (fixed summation orders).  Workspace: spai_logp_grad_workspace_bytes. */
size_t spai_logp_grad_workspace_bytes(int32_t E, int32_t T, int32_t B, int32_t per_sample);
int spai_logp_grad(const float* logits, int64_t bstride, int32_t E, int32_t B, const float* lmax,
                   const int64_t* actions, int64_t lda, int32_t T, const float* probs, int64_t ldp,
                   const float* gprobs, int64_t ldg, const uint32_t* removed, int32_t words, float* grad_out,
                   void* workspace, size_t workspace_bytes, void* stream);

/* BackwardPolicy's LSTM (policy.py:75-129; nn.LSTM(1, H), gate order i, f, g, o): input
 * x_t = (float)traj[b][t] for t < lengths[b] (the entries != -1, as pack_padded_sequence
 * takes them).  Forward: h_last [B][H] and, when states != NULL, what the backward needs in
 * states (spai_lstm_states_floats(B, H, T) floats): (h_t, c_t) of every step, [B][T][2H], for
 * H = 2, 8; for H = 4 the (h, c) checkpoint entering every 16-step block, [B][ceil(T/16)][2H]
 * (the backward recomputes the steps inside a block bit for bit).  Backward (BPTT from dh_last [B][H], dc = 0 at the end): one fp64 row
 * per sample in grad [B][4H + 4H*H + 4H] = d w_ih [4H] | d w_hh [4H][H] | d bias [4H]
 * (d b_ih = d b_hh = d bias).  H in {2, 4, 8}.  H = 4 runs the adjoint as a linear recurrence
 * over per-step coefficients kept in the workspace (spai_lstm_backward_workspace_bytes:
 * 288 B per (sample, step) + 48 KB per sample; 0 for H = 2, 8, where workspace may be NULL). */
size_t spai_lstm_backward_workspace_bytes(int32_t B, int32_t H, int32_t T);
size_t spai_lstm_states_floats(int32_t B, int32_t H, int32_t T);
int spai_lstm_forward(int32_t B, int32_t H, const int64_t* traj, int64_t ldt, const int32_t* lengths, int32_t T,
                      const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* h_last,
                      float* states, void* stream);
int spai_lstm_backward(int32_t B, int32_t H, const int64_t* traj, int64_t ldt, const int32_t* lengths, int32_t T,
                       const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                       const float* states, const float* dh_last, double* grad, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- rewards
 * residual[b] = sqrt(res2[b]) and reward[b] = 1000 * (alpha (1 - r/r0) + (1 - alpha)(1 - f/f0))
 * with f = 2 n (nnz0 - removed_counts[b]) (preconditioner.py:55-66, 68-77, 137-165; alpha is
 * the device fp32 scalar the rollout passes, not the never-set self.alpha of :163).  The
 * fp32/fp64 mix of the reference's torch type promotion is reproduced op for op.  reward32
 * (may be NULL) receives the fp32 copy Log.rewards holds (gflownet.py:193). */
int spai_rewards(const double* res2, const int32_t* removed_counts, int32_t B, int64_t nnz0, int32_t n,
                 double r0, double f0, const float* alpha, double* residual, double* reward, float* reward32,
                 void* stream);

/* ---------------------------------------------------------------- Krylov evaluation
 * y = A x (fp64 x, y; fp32 or fp64 values) over row-ELL lines idx/val [n][W] (-1 = padding),
 * slot order, fp64 fma: the products of GFlowNet100.py:61-93's GMRES (A v and the SPAI M v),
 * driven by gflownet_spai_amd/gmres.py. */
int spai_ell_spmv(int32_t n, int32_t W, const int32_t* idx, const void* val, int32_t val_dtype, const double* x,
                  double* y, void* stream);

/* ---------------------------------------------------------------- Matrix Market ingest (host)
 * gflownet/utils.py:54-63 market_matrix_to_sparse_tensor / GFlowNet100.py:44-46 load_mtx_file:
 * scipy.io.mmread(path).tocoo().  Coordinate format; field real / integer / pattern; symmetry
 * general / symmetric / skew-symmetric.  The COO written is mmread's entry for entry: the file
 * entries in file order (0-based), then the mirror (j, i) of every off-diagonal entry of a
 * (skew-)symmetric file in file order (value negated for skew), i.e. the raw order that defines
 * the action ids (preconditioner.py:23-25).  Host memory, no GPU.
 * spai_mtx_header: dims = {rows, cols, file entries, capacity spai_mtx_read needs},
 *                  kinds = {SPAI_MTX_REAL | _INTEGER | _PATTERN, SPAI_MTX_GENERAL | _SYMMETRIC | _SKEW}.
 * spai_mtx_read:   fills row/col (int64) and val (double), *nnz_out = entries written;
 *                  threads <= 0 = all hardware threads. */
#define SPAI_MTX_REAL 0
#define SPAI_MTX_INTEGER 1
#define SPAI_MTX_PATTERN 2
#define SPAI_MTX_GENERAL 0
#define SPAI_MTX_SYMMETRIC 1
#define SPAI_MTX_SKEW 2
int spai_mtx_header(const char* path, int64_t* dims, int32_t* kinds);
int spai_mtx_read(const char* path, int64_t* row, int64_t* col, double* val, int64_t capacity, int32_t threads,
                  int64_t* nnz_out);

#ifdef __cplusplus
}
#endif
#endif /* SPAI_HIP_H */
