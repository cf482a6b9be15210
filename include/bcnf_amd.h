/*
 * bcnf_amd — MI355X-native (gfx950 / CDNA4) CondRealNVP_v2 affine-coupling stack.
 *
 * C-ABI drop-in boundary for the reference's hot path (psaegert/bcnf, src/bcnf/models/cnf.py).
 * Plain pointers and sizes only; every tensor is fp32, row-major, contiguous, device-resident and
 * owned by the caller (the library holds no device memory across calls). Every entry point is
 * stream-ordered on the `stream` argument (a hipStream_t passed as void*), does not synchronise,
 * never throws, and returns BCNF_OK (0) or a nonzero status (see bcnf_status_string).
 *
 * The reference has no native code and hence no FFI; the functions below replace these
 * reference interfaces (file:line relative to /root/reference):
 *
 *   bcnf_stack_forward   <- CondRealNVP_v2.forward layer loop, cnf.py:476-488, with
 *                           ActNorm.forward cnf.py:348-351, ConditionalAffineCouplingLayer.forward
 *                           cnf.py:165-196 (nested MLP cnf.py:98-107) and OrthonormalTransformation.forward
 *                           cnf.py:333-335; log|det J| accumulation cnf.py:477,488; optional
 *                           log_prob = -inn_nll_loss(...,'none') - D/2 log 2pi (utils.py:49-53)
 *   bcnf_stack_backward  <- torch.autograd backward of the above (Trainer._train_batch, trainer.py:268)
 *   bcnf_stack_inverse   <- CondRealNVP_v2.inverse layer loop, cnf.py:499-506 (ActNorm.inverse
 *                           cnf.py:353-354, coupling inverse cnf.py:198-213, orthonormal inverse
 *                           cnf.py:337-339); with cond_index it also serves _sample's tiled
 *                           conditions (cnf.py:577-582) without materialising the tiled features
 *   bcnf_pack_params     <- (no reference counterpart) re-lays the nn.Module parameters into the
 *                           kernels' LDS-record layout; call after every parameter update
 *   bcnf_nll_forward     <- Trainer._train_batch forward + loss, trainer.py:260-266: the stack forward
 *                           fused with inn_nll_loss(z, log_det_J) (utils.py:40-46, reduction 'mean')
 *   bcnf_nll_backward    <- loss.backward() of that loss through the stack (trainer.py:268)
 *   bcnf_adam_step       <- optimizer.step() of torch.optim.Adam built by the Trainer (trainer.py:136,270)
 *   bcnf_clip_grad_norm  <- torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
 *                           (trainer.py:275, after the step)
 *   bcnf_linear_forward / bcnf_linear_backward
 *                        <- nn.Linear of FullyConnectedFeatureNetwork (feature_network.py:114-145)
 *   bcnf_wide_*          <- the same stack interfaces for the wide-MLP shapes (FC_large / LSTM_large)
 *   bcnf_rank_count      <- the rank count of compute_y_hat_ranks (eval/calibration.py:42-46)
 *   bcnf_resimulate      <- resimulate's per-draw physics_ODE_simulation map (simulation/resimulation.py:12-18,
 *                           49-56 -> simulation/physics.py:53-160)
 */
#ifndef BCNF_AMD_H
#define BCNF_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCNF_MAX_HIDDEN 8
#define BCNF_MAX_TENSORS 48
/* Layout version of the structs below (2: BcnfStackDesc.gemm_tiling appended). bcnf_abi_version() returns the
 * library's; a caller compares it with this macro before passing any struct. */
#define BCNF_AMD_ABI_VERSION 2

int bcnf_abi_version(void);

enum {
  BCNF_OK = 0,
  BCNF_ERR_ARG = 1,          /* invalid descriptor / null pointer / bad size */
  BCNF_ERR_UNSUPPORTED = 2,  /* shape outside this kernel family (see bcnf_stack_supported) */
  BCNF_ERR_HIP = 3           /* reserved (a HIP failure returns BCNF_ERR_HIP_BASE + its hipError_t)       */
};
/* A HIP runtime failure (launch, attribute, memset / copy) returns BCNF_ERR_HIP_BASE + the hipError_t it produced;
 * bcnf_status_string names it. The library keeps no error state between calls. */
#define BCNF_ERR_HIP_BASE 1000

/* Mirrors CondRealNVP_v2.__init__ kwargs (cnf.py:358-375) for the coupling stack. */
typedef struct BcnfStackDesc {
  int32_t size;                      /* D                                     */
  int32_t n_conditions;              /* C (features per sample, h.shape[1])   */
  int32_t n_hidden;                  /* len(nested_sizes)                      */
  int32_t hidden[BCNF_MAX_HIDDEN];   /* nested_sizes                           */
  int32_t n_blocks;                  /* n_blocks                               */
  int32_t act_norm;                  /* 0/1                                    */
  int32_t two_way;                   /* 0/1 (small family: 0 only; wide: both) */
  float dropout;                     /* p of every nn.Dropout in the nested MLP */
  int32_t gemm_tiling;               /* wide family only: 0 = each GEMM's cost-model tiling (use this); t + 1 forces
                                        tiling t (0 <= t <= 10, see bcnf_wide_gemm_test) on every GEMM of the call
                                        (tests / A-B timing). Per call: the library holds no such setting. Appended
                                        in ABI version 2 (BCNF_AMD_ABI_VERSION): C callers built against a version-1
                                        header pass a shorter struct and must be rebuilt. */
} BcnfStackDesc;

/* 1 if this descriptor runs on the fused small-width kernel family, else 0. */
int bcnf_stack_supported(const BcnfStackDesc* desc);

/* Canonical flat layouts (state_dict order of layers.*, frozen orthonormal matrices excluded /
 * separate): n_trainable = #floats of ActNorm + coupling params, n_frozen = (n_blocks-1)*D*D. */
int bcnf_param_count(const BcnfStackDesc* desc, int64_t* n_trainable, int64_t* n_frozen);

/* Bytes of the packed-parameter buffer written by bcnf_pack_params. */
int bcnf_packed_bytes(const BcnfStackDesc* desc, int64_t* bytes);

/* Bytes of the forward->backward workspace for a batch: saved block inputs, dropout masks, loss
 * partials, the hoisted condition projection HP[k][b][16] = h W1h_k^T + b1_k and the Linear-1 deltas
 * D1[k][b][16] written by the backward. Required by every forward and backward call. */
int bcnf_workspace_bytes(const BcnfStackDesc* desc, int64_t batch, int32_t training, int64_t* bytes);

/* Bytes of the gradient scratch ("slab") of a backward over `batch` samples: per-workgroup partial
 * gradients plus the split-K partials of the W1 condition columns. */
int bcnf_slab_bytes(const BcnfStackDesc* desc, int64_t batch, int64_t* bytes);

/* Bytes of the inverse's scratch (the condition projection of h_rows feature rows). */
int bcnf_inverse_scratch_bytes(const BcnfStackDesc* desc, int64_t h_rows, int64_t* bytes);

/* Re-lay params (canonical flat, n_trainable floats) and qmats ((n_blocks-1)*D*D floats) into
 * `packed` (bcnf_packed_bytes). Also writes the ActNorm log|det| constant used by the forward. */
int bcnf_pack_params(const BcnfStackDesc* desc, const float* params, const float* qmats, void* packed,
                     void* stream);

/* Forward of the whole stack given features h (B x C): z (B x D), ldj (B), optional log_prob (B).
 * training != 0 applies dropout with the counter-based RNG keyed by rng_state[0] (seed) and
 * rng_state[1] (offset), both read from DEVICE memory (graph-replay safe). `workspace`
 * (bcnf_workspace_bytes) is required; save != 0 also keeps what bcnf_stack_backward needs. */
int bcnf_stack_forward(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h,
                       int64_t batch, float* z, float* ldj, float* log_prob, int32_t training,
                       const uint64_t* rng_state, void* workspace, int32_t save, void* stream);

/* Backward: given dz (B x D) and dldj (B) (either may be NULL = zeros), writes dh (B x C,
 * overwritten, nullable), dy (B x D, nullable) and the gradient scratch `slab` (bcnf_slab_bytes).
 * With dparams != NULL it then reduces into dparams (canonical flat, n_trainable floats, overwritten);
 * with dparams == NULL the caller runs bcnf_grad_reduce. `training` and `workspace` must be those of
 * the (save != 0) forward call. */
int bcnf_stack_backward(const BcnfStackDesc* desc, const void* packed, const float* h, const float* dz,
                        const float* dldj, int64_t batch, int32_t training, void* workspace, float* dy,
                        float* dh, float* dparams, void* slab, void* stream);

/* dL/dh (B x C, overwritten) = sum_k D1_k W1h_k from the deltas a backward left in `workspace` (what
 * bcnf_stack_backward does itself when its dh != NULL). */
int bcnf_stack_dh(const BcnfStackDesc* desc, const void* packed, const void* workspace, int64_t batch,
                  int32_t training, float* dh, void* stream);

/* Everything after bcnf_stack_backward(dh = dparams = NULL) in one go: dh (nullable) and dparams, as
 * bcnf_stack_dh + bcnf_grad_reduce but with the independent pieces sharing one launch. */
int bcnf_backward_tail(const BcnfStackDesc* desc, const void* packed, const void* slab, const float* h,
                       const void* workspace, int64_t batch, int32_t training, float* dh, float* dparams,
                       void* stream);

/* ---- Folded linear feature network (training fast path; no reference counterpart as a function: it
 * computes the same sums as feature_network.py:114-145's single nn.Linear [X -> C] feeding cnf.py:74-107's
 * condition input, reassociated). With Wf (C x X, row-major) and bf (C, nullable) of that Linear:
 *   Wc = W1h Wf, bc = b1 + W1h bf  (bcnf_pack_params_fold, alongside the training sections of the regular pack
 *                                   -- forward / backward records, W1hR, log-det constant; NOT the inverse records,
 *                                   so its `packed` serves the folded training pass only -- one launch)
 *   HP = x Wc^T + bc               (bcnf_fold_nll_forward: bcnf_nll_forward with x (B x X) in place of h)
 *   dW1h, dWf, dbf from Gx = D1^T [x | 1]  (bcnf_fold_backward_tail, after bcnf_nll_backward(dh = dparams
 *   = NULL) wrote `slab` sized by bcnf_fold_slab_bytes). h and dL/dh are never formed. X + 1 <= 256.
 * x rows are ldx >= X floats apart; ldx % 4 == 0 with a 16-byte aligned x selects float4 row loads (TrainStep's
 * padded pool, bcnf_amd/train.py); the padding columns are never used. */
int bcnf_fold_bytes(const BcnfStackDesc* desc, int32_t in_features, int64_t* bytes);
int bcnf_fold_slab_bytes(const BcnfStackDesc* desc, int32_t in_features, int64_t batch, int64_t* bytes);
/* A batch gather to run inside bcnf_pack_params_fold's launch (the pack does not read the batch, so the two are
 * independent): the arguments of bcnf_gather_rows2 (cursor = NULL) or bcnf_gather_batch (idx = the epoch order). */
typedef struct BcnfGather2 {
  const int64_t* idx;
  const int64_t* cursor;
  int64_t n;
  const float* src0;
  int32_t cols0;
  float* dst0;
  const float* src1;
  int32_t cols1;
  float* dst1;
} BcnfGather2;
int bcnf_pack_params_fold(const BcnfStackDesc* desc, const float* params, const float* qmats,
                          const float* feat_weight, const float* feat_bias, int32_t in_features, void* packed,
                          float* fold, const BcnfGather2* gather /* nullable */, void* stream);
int bcnf_fold_nll_forward(const BcnfStackDesc* desc, const void* packed, const float* fold, int32_t in_features,
                          const float* y, const float* x, int32_t ldx, int64_t batch, float* z, float* ldj,
                          int32_t training,
                          uint64_t* rng_state, void* workspace, int32_t finalize, float* loss_out, int32_t* guard,
                          void* stream);
/* Pack-free folded training forward: bcnf_pack_params_fold + bcnf_fold_nll_forward in ONE launch. The
 * forward builds its records from `params` / `qmats` through a per-layout table (bcnf_fold_raw_table, built once on
 * the host and copied to the device by the caller), computes h = x Wf^T + bf of its rows on the matrix cores and the
 * condition projection from h (the unfolded sums, so the loss rounds like bcnf_nll_forward on h rather than like the
 * folded Wc), and writes into `packed` exactly what bcnf_nll_backward + bcnf_fold_backward_tail read (backward
 * records, W1hR) -- `packed` serves that training pass only. gather (nullable): the rows come from the pools
 * (src0 [*][D], src1 [*][cols1]; n == batch), y / x are then unused and the forward writes the gathered rows into
 * dst0 / dst1 (ldx = cols1), as bcnf_pack_params_fold's gather did. BCNF_ERR_UNSUPPORTED where the table does not
 * apply (no ActNorm, one block, X > 128) -- use the two-launch form there. bcnf_fold_raw_table_bytes: the table's
 * size in bytes; bcnf_fold_raw_table fills `host_table` (host memory) with it. */
int bcnf_fold_raw_table_bytes(const BcnfStackDesc* desc, int32_t in_features, int64_t* bytes);
int bcnf_fold_raw_table(const BcnfStackDesc* desc, int32_t in_features, void* host_table);
int bcnf_fold_train_forward(const BcnfStackDesc* desc, const float* params, const float* qmats, const void* table,
                            const float* feat_weight, const float* feat_bias, int32_t in_features,
                            const BcnfGather2* gather /* nullable */, const float* y, const float* x, int32_t ldx,
                            int64_t batch, void* packed, float* z, float* ldj, int32_t training,
                            uint64_t* rng_state, void* workspace, int32_t finalize, float* loss_out, int32_t* guard,
                            void* stream);
/* Adam fused into bcnf_fold_backward_tail (nullable argument): every gradient the tail produces -- the flat coupling
 * parameters (slot 0), the feature Linear's weight (1) and bias (2, NULL without bias) -- also takes its
 * torch.optim.Adam update where it is produced, with the end-of-step bookkeeping of bcnf_adam_step_bookkeep
 * (step count, epoch cursor, logged values; done_counter: device int32, 0 between launches). For a training step
 * whose clip-after-step cannot be observed (trainer.py:273-275; see bcnf_adam_step_bookkeep): it replaces that
 * step's Adam launch. The gradients are still written. */
typedef struct BcnfFoldAdam {
  float* params[3];
  float* exp_avg[3];
  float* exp_avg_sq[3];
  float* step;
  double lr, beta1, beta2, eps, weight_decay;
  int64_t* advance_cursor;
  int64_t cursor_modulo;
  const float* log_values;
  float* log_history;
  int32_t* done_counter;
  const int32_t* guard;
} BcnfFoldAdam;
int bcnf_fold_backward_tail(const BcnfStackDesc* desc, const void* packed, const void* slab, const float* x,
                            int32_t ldx, int32_t in_features, const float* feat_weight, const float* feat_bias,
                            const void* workspace, int64_t batch, int32_t training, float* dparams,
                            float* dfeat_weight, float* dfeat_bias, const BcnfFoldAdam* adam /* nullable */,
                            void* stream);

/* Deterministic (fixed-order) reduction of a backward's gradient scratch into dparams, including the
 * W1 condition columns (split-K GEMM of D1 with h). Replaces autograd's implicit batch reduction. */
int bcnf_grad_reduce(const BcnfStackDesc* desc, const void* slab, const float* h, const void* workspace,
                     int64_t batch, int32_t training, float* dparams, void* stream);

/* Inverse of the whole stack: y (N x D) from z (N x D). h has h_rows rows; row r uses feature row
 * cond_index[r] when cond_index != NULL (h_rows may then be anything), else row r (h_rows == N).
 * `scratch`: bcnf_inverse_scratch_bytes(h_rows) -- the projection is computed once per feature row.
 * Without dropout (eval, or p = 0) the stack runs on the matrix cores, 16 rows per wave;
 * training mode with dropout keeps the row-layout kernel. A row's result does not depend on its position. */
int bcnf_stack_inverse(const BcnfStackDesc* desc, const void* packed, const float* z, const float* h,
                       int64_t h_rows, const int64_t* cond_index, int64_t n_rows, float* y, int32_t training,
                       const uint64_t* rng_state, void* scratch, void* stream);

/* ---- NLL training pass (forward + inn_nll_loss + backward without any host round trip) ---------
 * bcnf_nll_forward = bcnf_stack_forward (workspace required, save on) plus per-workgroup partials of
 *   nll = mean_b(0.5 |z_b|^2 - ldj_b)  (utils.py:40-46). With finalize != 0 a one-workgroup launch then
 *   writes loss_out[0] = loss = (nll + 0 * mse) / (1 + 0), loss_out[1] = nll, loss_out[2] = mse = 0 (the
 *   Trainer's three logged values with hybrid_weight == 0) and, when dropout is active, advances
 *   rng_state[1] by one (so graph replays draw fresh masks). With finalize == 0 that reduction is
 *   deferred to bcnf_nll_backward(loss_out, rng_state) (saves a launch in a training step). No kernel
 *   synchronises across workgroups. */
int bcnf_nll_forward(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h, int64_t batch,
                     float* z, float* ldj, int32_t training, uint64_t* rng_state, void* workspace, int32_t finalize,
                     float* loss_out, int32_t* guard, void* stream);

/* Backward through loss_out w.r.t. y, h and the stack parameters: dz = z * g / B, dldj = -g / B with
 * g = dloss[0] + dloss[1], dloss being the device cotangent of loss_out[0..2] (NULL means d loss = 1,
 * i.e. loss.backward(); mse carries no gradient). z is the forward's output. With loss_out != NULL it
 * also performs the forward's deferred loss reduction (finalize == 0 there). Otherwise as
 * bcnf_stack_backward. */
int bcnf_nll_backward(const BcnfStackDesc* desc, const void* packed, const float* h, const float* z,
                      const float* dloss, int64_t batch, int32_t training, void* workspace, float* dy,
                      float* dh, float* dparams, void* slab, float* loss_out, uint64_t* rng_state, int32_t* guard,
                      void* stream);

/* ---- Optimizer ------------------------------------------------------------------------------------
 * Tensors are passed as arrays of n_tensors (<= BCNF_MAX_TENSORS) device pointers + element counts and
 * treated as one concatenated index space. bcnf_grad_partials(total) = floats of the partials buffer the kernels
 * below write / read: one sum of squared gradients per workgroup, plus one slot for their pre-reduced total. */
int64_t bcnf_grad_partials(int64_t total_numel);

/* One torch.optim.Adam step (amsgrad = maximize = False) over every tensor; hyper-parameters are
 * doubles (derived scalars such as 1 - beta2 are formed in double and rounded once, as torch does);
 * `step` is the device-side float step count (as Adam(capturable=True) keeps it): the update uses
 * step + 1, and advance_step != 0 then stores it (a one-thread launch). With advance_step == 0 the
 * caller advances it later (bcnf_clip_grad_norm(advance_step = step)), saving that launch. With
 * grad_partials != NULL the per-workgroup sums of squared gradients for bcnf_clip_grad_norm are written. */
int bcnf_adam_step(int32_t n_tensors, float* const* params, float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numel, float* step, double lr, double beta1,
                   double beta2, double eps, double weight_decay, float* grad_partials, int32_t advance_step,
                   const int32_t* guard, void* stream);

/* bcnf_adam_step (step count advanced in the same launch) whose LAST workgroup to finish also does the end-of-step
 * bookkeeping of bcnf_clip_grad_norm: epoch cursor advance and logged values -> log_history[3 * cursor]. It
 * replaces Adam + clip for a training step whose clip-after-step (trainer.py:275) cannot be observed -- one that
 * is followed, inside the same captured graph, by the next step's backward, which overwrites every gradient the
 * clip would scale (the reference discards the returned norm). done_counter: device int32, 0 between launches
 * (the last workgroup resets it). No squared-gradient partials are written. */
int bcnf_adam_step_bookkeep(int32_t n_tensors, float* const* params, float* const* grads, float* const* exp_avg,
                            float* const* exp_avg_sq, const int64_t* numel, float* step, double lr, double beta1,
                            double beta2, double eps, double weight_decay, int64_t* advance_cursor,
                            int64_t cursor_modulo, const float* log_values, float* log_history, int32_t* done_counter,
                            const int32_t* guard, void* stream);

/* Per-workgroup sums of squared gradients (when no bcnf_adam_step produced them). */
int bcnf_grad_sumsq(int32_t n_tensors, float* const* grads, const int64_t* numel, float* grad_partials, void* stream);

/* clip_grad_norm_(max_norm, norm_type=2): total = sqrt(sum partials); g *= min(max_norm/(total+1e-6), 1).
 * total_norm (device float, nullable) receives the pre-clip norm. End-of-step bookkeeping (nullable):
 * advance_step[0] += 1 (a deferred Adam step count) and advance_cursor[0] = (cursor + 1) % cursor_modulo
 * (an epoch cursor of bcnf_gather_batch). */
int bcnf_clip_grad_norm(int32_t n_tensors, float* const* grads, const int64_t* numel, const float* grad_partials,
                        float max_norm, float* total_norm, float* advance_step, int64_t* advance_cursor,
                        int64_t cursor_modulo, const float* log_values, float* log_history, const int32_t* guard,
                        void* stream);

/* Training-loop guard, int32[4] in device memory (nullable everywhere): [BCNF_GUARD_CHECK] is set by the
 * host (the Trainer checks for divergence after epoch 10, trainer.py:168); the loss finalize of
 * bcnf_nll_forward / bcnf_nll_backward raises [BCNF_GUARD_DIVERGED] when loss > 1e5 or NaN and, one step
 * later, [BCNF_GUARD_HALTED], which makes that step's RNG advance, bcnf_adam_step and bcnf_clip_grad_norm
 * no-ops. Steps can so be replayed back to back without a host sync per step: the host reads the logged
 * values afterwards and raises where the reference would, with the state it would have had.
 * bcnf_clip_grad_norm also stores log_values[0..2] (the step's loss, nll, mse) into
 * log_history[3 * cursor ...] (cursor = advance_cursor[0] before the advance, else 0); log_history may be
 * pinned host memory (system-scope stores). */
#define BCNF_GUARD_CHECK 0
#define BCNF_GUARD_DIVERGED 1
#define BCNF_GUARD_HALTED 2
#define BCNF_GUARD_CHECK_GLOBAL 3
#define BCNF_GUARD_WORDS 4

/* Data parallel form of the divergence check (trainer.py:168 on the loss every rank logs): the host leaves
 * [BCNF_GUARD_CHECK] at 0, so no rank's loss finalize judges its local shard, and sets
 * [BCNF_GUARD_CHECK_GLOBAL]; after the gradient all-reduce this one-thread launch raises [BCNF_GUARD_DIVERGED]
 * when the all-reduced loss global_values[0] > 1e5 or NaN (unless the step is already halted). Every rank sees
 * the same value, so every rank halts on the same step; the next step's loss finalize turns DIVERGED into
 * HALTED exactly as in the single-process case. */
int bcnf_guard_check_global(const float* global_values, int32_t* guard, void* stream);

/* The same bookkeeping as a one-thread launch. */
int bcnf_advance_counters(float* step, int64_t* cursor, int64_t n_batches, void* stream);

/* ---- Batch feed: dst0[r] = src0[idx[r]], dst1[r] = src1[idx[r]] (row-major rows of cols0 / cols1
 * floats) in one launch -- the shuffled-batch gather of the Trainer's DataLoader (trainer.py:164-166)
 * from device-resident data. */
int bcnf_gather_rows2(const int64_t* idx, int64_t n, const float* src0, int32_t cols0, float* dst0,
                      const float* src1, int32_t cols1, float* dst1, void* stream);
/* The same for batch number cursor[0] of an epoch order (device int64 indices, batch per batch): rows
 * order[cursor[0] * batch + r]. The cursor is advanced by a later launch (bcnf_clip_grad_norm /
 * bcnf_advance_counters), so the gather needs no cross-workgroup synchronisation (graph-replay safe). */
int bcnf_gather_batch(const int64_t* order, const int64_t* cursor, int64_t batch, const float* src0, int32_t cols0,
                      float* dst0, const float* src1, int32_t cols1, float* dst1, void* stream);

/* ---- nn.Linear (row-major, weight out_features x in_features) ------------------------------------ */
int bcnf_linear_forward(const float* x, const float* weight, const float* bias, int64_t rows, int32_t in_features,
                        int32_t out_features, float* y, void* stream);
/* Scratch bytes bcnf_linear_backward needs for its split-K weight gradient. */
int64_t bcnf_linear_work_bytes(int64_t rows, int32_t in_features, int32_t out_features);
/* dx (nullable) = dy W; dweight = dy^T x and dbias (nullable) = column sums of dy, both overwritten
 * (fixed-order split-K reduction through `work`). dweight may be NULL only when dbias is NULL too. */
int bcnf_linear_backward(const float* x, const float* weight, const float* dy, int64_t rows, int32_t in_features,
                         int32_t out_features, float* dx, float* dweight, float* dbias, void* work, void* stream);
/* One hidden layer of a FullyConnectedFeatureNetwork, nn.Linear -> nn.GELU() -> nn.Dropout(p) (feature_network.py:
 * 128-134, the reference runs them as three ATen ops), in ONE launch: a = mask GELU(x W^T + b) with the exact-erf
 * GELU, and g (nullable) = mask GELU'(x W^T + b) for the backward. mask = 1 / (1 - p) or 0 from an in-kernel
 * Philox4x32-10 stream when rng (device uint64 [seed, offset], read only) is given and p > 0, else 1; salt separates
 * the layers of one network. Same element-wise distribution as torch's dropout, not its bits. */
int bcnf_linear_gelu_forward(const float* x, const float* weight, const float* bias, int64_t rows, int32_t in_features,
                             int32_t out_features, float p, const uint64_t* rng, int32_t salt, float* a, float* g,
                             void* stream);
/* Backward of bcnf_linear_gelu_forward from dL/da and its g: dL/dpre = da * g is formed as the operands are loaded
 * (never stored), then as bcnf_linear_backward (same work bytes). */
int bcnf_linear_gelu_backward(const float* x, const float* weight, const float* da, const float* g, int64_t rows,
                              int32_t in_features, int32_t out_features, float* dx, float* dweight, float* dbias,
                              void* work, void* stream);

/* ---- Wide-MLP family (trajectory_FC_large / trajectory_LSTM_large class: nested_sizes = [H] * NH with H too
 * wide for the register-resident kernels above, e.g. [526] * 5, C = 1360, 26 blocks) ----------------------------
 * Same BcnfStackDesc, same canonical flat parameter layout (state_dict order) and the same reference interfaces
 * as bcnf_stack_forward / _backward / _inverse / bcnf_nll_* above (cnf.py:49-107, 165-213, 312-354, 467-508;
 * utils.py:40-53; trainer.py:260-268), built from fp32-MFMA GEMMs (v_mfma_f32_32x32x2_f32) with fused
 * bias / GELU / dropout / gradient epilogues and per-sample link kernels (coupling, log|det J|, orthonormal mix,
 * ActNorm). Requirements: equal nested sizes, size <= 32. two_way couplings (cnf.py:176-186) run as two
 * half-couplings per block (nn_a then nn_b), with the reference's inverse (cnf.py:198-213).
 * The wide family takes the canonical flat params directly plus its own packed buffer (padded weight copies,
 * bcnf_wide_pack after every parameter update). */
int bcnf_wide_supported(const BcnfStackDesc* desc);
/* Canonical flat sizes as bcnf_param_count, for the wide family (two_way: nn_a then nn_b per block). */
int bcnf_wide_param_count(const BcnfStackDesc* desc, int64_t* n_trainable, int64_t* n_frozen);
int bcnf_wide_packed_bytes(const BcnfStackDesc* desc, int64_t* bytes);
/* save != 0: the forward keeps every activation, GELU-derivative factor and block input for the backward. */
int bcnf_wide_workspace_bytes(const BcnfStackDesc* desc, int64_t batch, int32_t save, int64_t* bytes);
int bcnf_wide_inverse_scratch_bytes(const BcnfStackDesc* desc, int64_t h_rows, int64_t n_rows, int64_t* bytes);
int bcnf_wide_pack(const BcnfStackDesc* desc, const float* params, const float* qmats, void* packed, void* stream);
/* z (B x D), ldj (B); nll_part (nullable) receives 0.5 |z_b|^2 - ldj_b per sample (the per-sample inn_nll_loss,
 * utils.py:49-53 with reduction 'none'). Dropout as bcnf_stack_forward (device rng_state; the caller advances the
 * offset, or bcnf_wide_nll_finalize does). */
int bcnf_wide_forward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* y,
                      const float* h, int64_t batch, float* z, float* ldj, float* nll_part, int32_t training,
                      const uint64_t* rng_state, void* workspace, int32_t save, void* stream);
/* loss_out[0..2] = [loss, nll, mse = 0] from the forward's per-sample NLL terms (workspace of that forward), plus
 * the dropout RNG advance and the divergence guard, as bcnf_nll_forward's finalize. */
int bcnf_wide_nll_finalize(const BcnfStackDesc* desc, const void* workspace, int64_t batch, int32_t save,
                           float* loss_out, uint64_t* rng_state, int32_t* guard, void* stream);
/* Backward of a save != 0 forward. nll == 0: cotangents dz (B x D) / dldj (B), either nullable. nll != 0: through
 * the NLL, dz = z g / B and dldj = -g / B with g = dloss[0] + dloss[1] (dloss nullable = 1), z = the forward's
 * output. Writes dy, dh (nullable) and dparams (canonical flat, every element overwritten; nullable). */
int bcnf_wide_backward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* h,
                       const float* z, const float* dz, const float* dldj, const float* dloss, int32_t nll,
                       int64_t batch, void* workspace, float* dy, float* dh, float* dparams, void* stream);
/* Folded last feature Linear of a wide stack (trajectory_FC_large: h = x Wf^T + bf, feature_network.py:114-145 with
 * the stack's condition projection cnf.py:98-107): with x1 = [x | 1 | 0] (B x xp, xp = roundup(X + 1, 4), 16-B
 * aligned rows), wfb = [Wf | bf | 0] (C x xp) and Wcb = W0h_all wfb (nv*HP x xp):
 *   prepare:  Wcb = W0h_all wfb (after bcnf_wide_pack; wcb holds nv*HP*xp floats, nv*HP = bcnf_wide_param_count's
 *             layout: blocks x sides x 16-padded hidden width)
 *   forward:  P = x1 Wcb^T, then the unchanged stack (save is implied: a backward follows)
 *   backward: through the NLL (dloss nullable = 1): Gx = dZ0^T x1 (gx_scratch, nv*HP*xp floats), dW0h = Gx wfb^T
 *             into dparams, dwfb = W0h_all^T Gx (C x xp: [dWf | dbf]), dx = dZ0 Wcb (B x xp, columns < X).
 * h and dL/dh are never formed. */
int bcnf_wide_fold_prepare(const BcnfStackDesc* desc, const void* packed, const float* wfb, int32_t xp, float* wcb,
                           void* stream);
int bcnf_wide_fold_forward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* y,
                           const float* x1, int32_t xp, const float* wcb, int64_t batch, float* z, float* ldj,
                           int32_t training, const uint64_t* rng_state, void* workspace, void* stream);
int bcnf_wide_fold_backward(const BcnfStackDesc* desc, const float* params, const void* packed, const float* x1,
                            int32_t xp, const float* wfb, const float* wcb, const float* z, const float* dloss,
                            int64_t batch, void* workspace, float* gx_scratch, float* dparams, float* dwfb, float* dx,
                            void* stream);
/* bcnf_wide_fold_backward split over real blocks, for data parallelism that overlaps the gradient exchange with the
 * rest of the backward (trainer.py:244-277 is the single-process step it splits): one call per
 * contiguous block range [block_lo, block_hi), in descending order over one forward's workspace, the first with
 * block_hi = nb and the last with block_lo = 0. A call runs the backward chain until blocks [block_lo, block_hi) are
 * complete and writes their canonical parameter gradients, dparams[bcnf_wide_block_offset(block_lo) ..
 * bcnf_wide_block_offset(block_hi)); the block_lo = 0 call also writes dwfb and dx. Results equal one
 * bcnf_wide_fold_backward call bit for bit; calls out of that order leave the outputs undefined. */
int bcnf_wide_fold_backward_range(const BcnfStackDesc* desc, const float* params, const void* packed, const float* x1,
                                  int32_t xp, const float* wfb, const float* wcb, const float* z, const float* dloss,
                                  int64_t batch, void* workspace, float* gx_scratch, float* dparams, float* dwfb,
                                  float* dx, int32_t block_lo, int32_t block_hi, void* stream);
/* bcnf_wide_fold_backward in two phases, for a caller that overlaps the coupling parameter gradients with the rest of
 * its own backward (the feature network's, trainer.py:244-277 runs both in one loss.backward()): phase 1 writes dx and
 * dwfb (and gx_scratch), phase 2 writes dparams; phase 2 must follow phase 1 in stream order (a second stream waiting
 * on an event recorded after phase 1 is the intended use) and both must finish before the next call on the same
 * workspace. phase 3 = both, one stream. Results equal one bcnf_wide_fold_backward call bit for bit. */
int bcnf_wide_fold_backward_phase(const BcnfStackDesc* desc, const float* params, const void* packed, const float* x1,
                                  int32_t xp, const float* wfb, const float* wcb, const float* z, const float* dloss,
                                  int64_t batch, void* workspace, float* gx_scratch, float* dparams, float* dwfb,
                                  float* dx, int32_t phase, void* stream);
/* Canonical flat offset of real block `block`'s first trainable parameter (its ActNorm, cnf.py:296-335 module order);
 * block = nb gives the parameter count. Host-only. */
int bcnf_wide_block_offset(const BcnfStackDesc* desc, int32_t block, int64_t* offset);
/* Rows of the padded projection (nv*HP) of a wide stack. */
int bcnf_wide_proj_rows(const BcnfStackDesc* desc, int64_t* rows);
/* Inverse: as bcnf_stack_inverse (cond_index selects feature rows; scratch = bcnf_wide_inverse_scratch_bytes). */
int bcnf_wide_inverse(const BcnfStackDesc* desc, const float* params, const void* packed, const float* z,
                      const float* h, int64_t h_rows, const int64_t* cond_index, int64_t n_rows, float* y,
                      int32_t training, const uint64_t* rng_state, void* scratch, void* stream);
/* ---- Calibration (eval/calibration.py:20-48, compute_y_hat_ranks) -----------------------------------------------
 * counts[i * dim + d] += #{ s < n_draws : y_hat[(s * n_rows + i) * dim + d] < y[i * dim + d] } for the (n_draws, n_rows,
 * dim) draws of sample(outer=True); counts is uint32 and accumulates, so draws can be fed in chunks. */
int bcnf_rank_count(const float* y_hat, const float* y, int64_t n_draws, int64_t n_rows, int32_t dim, uint32_t* counts,
                    void* stream);

/* ---- Re-simulation (simulation/resimulation.py:21-59 -> physics.py:53-160, physics_ODE_simulation per draw) -------
 * Replaces the ProcessPoolExecutor map of resimulate_trajectory (resimulation.py:12-18, 49-56) over every (draw j,
 * trajectory i). Physics parameter q (physics.py:53-72 order: x0_x x0_y x0_z v0_x v0_y v0_z g_x g_y g_z w_x w_y w_z
 * b m rho r a_x a_y a_z) is y_hat[(j * n_traj + i) * dim + param_cols[q]] (float32, or float64 with y_hat_f64) when
 * param_cols[q] >= 0 (the model predicts it: ParameterIndexMapping.dictify), else fixed[i * 19 + q] (the trajectory's
 * data_dict value, resimulation.py:53). tgrid = np.arange(0, T, dt) (steps >= 1 entries). Output
 * x[((i * n_draws + j) * steps + s) * 3 + c] (float64, = np.array(X_resimulation_list)). The velocity ODE is
 * integrated in fp64 by an adaptive Dormand-Prince 5(4) pair at (rtol, atol) between grid times; max_attempts bounds
 * the step attempts per trajectory. param_cols is a HOST array of 19; every other pointer is device memory.
 * attempts / status (int32 per (i, j)) are optional; status is BCNF_RESIM_*; a
 * trajectory that is not OK is NaN from the first grid time it could not reach. */
#define BCNF_RESIM_NPARAM 19
#define BCNF_RESIM_OK 0
#define BCNF_RESIM_NONFINITE 1   /* non-finite right-hand side at t = 0 (e.g. zero wind: 0/0 in physics.py:42) */
#define BCNF_RESIM_STEPS 2       /* step size underflow or max_attempts exhausted (divergent draw) */
int bcnf_resimulate(const void* y_hat, int32_t y_hat_f64, int64_t n_draws, int64_t n_traj, int32_t dim,
                    const int32_t* param_cols, const double* fixed, const double* tgrid, int32_t steps, double dt,
                    int32_t break_on_impact, double rtol, double atol, int32_t max_attempts, double* x,
                    int32_t* attempts, int32_t* status, void* stream);


const char* bcnf_status_string(int status);

/* ---------------------------------------------------------------------------------------------------------------
 * TEST-ONLY entry points. Not part of the drop-in boundary (no reference interface maps to them; INTEGRATION.md
 * binds none of them): exported so the GPU tests can poison LDS and exercise single GEMM tilings through ctypes.
 * ------------------------------------------------------------------------------------------------------------- */
/* Test hook (no reference counterpart): fill every CU's LDS with `value` (one full-LDS workgroup per CU, several
 * rounds), so a test can check that a following launch never reads LDS it did not write (the pack-free forward's
 * K padding, tests/test_gpu_fold.py). */
int bcnf_lds_fill(float value, void* stream);
/* Test hook for the GEMM tiles: C (M x N) = A B with (layout & 15) 0 = A[m][k] B[n][k], 1 = A[m][k] B[k][n],
 * 2 = A[k][m] B[k][n], 3 = A[k][m] B[n][k]; layout >> 4 forces a tiling as BcnfStackDesc.gemm_tiling (0 = the
 * dispatcher's choice, t + 1 = tiling t: 0 = 128x128 and 1 = 64x64 on v_mfma_f32_32x32x2_f32, 2 = 128x48, 3 = 128x48
 * on 8 waves, 4 = 96x48 on 6 waves (v_mfma_f32_16x16x4_f32), 5 / 6 / 7 = LDS-DMA tiling C auto / large / 48x48,
 * 8 = 176x176 on 11 waves (strided x strided layouts only), 9 / 10 = tiling W 96x48 / 48x48 (layout 0 only, the B band
 * resident in LDS, K <= 768); a forced tiling that does not apply to the layout / K runs as 64x64 (tiling 1);
 * leading dimensions and K multiples of 4, 16-byte aligned bases. Strided operands ([K][M] / [K][N] rows) are read
 * as whole float4 up to roundup4(M) / roundup4(N) columns in EVERY row, the last one included: allocate K * ld
 * floats for them (a tight (K - 1) * ld + M buffer is read out of bounds). */
int bcnf_wide_gemm_test(int32_t layout, int32_t M, int32_t N, int32_t K, const float* A, int64_t lda, const float* B,
                        int64_t ldb, float* C, int64_t ldc, void* stream);
/* Test hook (host arithmetic only, no launch): the workspace / G-region plan of one folded wide backward call
 * (bcnf_wide_fold_backward_range) at `batch` rows over blocks [block_lo, block_hi), dL/dx and [dWf | dbf] wanted or
 * not: out[0] = training workspace floats, out[1] = offset of the G region in it, out[2] = G region floats, out[3] =
 * the feature-side split-K partials at the region's end, out[4] / out[5] = offset (within G) / floats of the range's
 * parameter-gradient split-K scratch, out[6] / out[7] = the dL/dx / [dWf | dbf] partial needs. Checked by
 * tests/test_native_abi.py and under AddressSanitizer (tools/asan_host.sh). */
int bcnf_wide_backward_plan(const BcnfStackDesc* desc, int64_t batch, int32_t xp, int32_t want_dx, int32_t want_dwfb,
                            int32_t block_lo, int32_t block_hi, int64_t* out);

#ifdef __cplusplus
}
#endif

#endif /* BCNF_AMD_H */
