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
 */
#ifndef BCNF_AMD_H
#define BCNF_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCNF_MAX_HIDDEN 8

enum {
  BCNF_OK = 0,
  BCNF_ERR_ARG = 1,          /* invalid descriptor / null pointer / bad size */
  BCNF_ERR_UNSUPPORTED = 2,  /* shape outside this kernel family (see bcnf_stack_supported) */
  BCNF_ERR_HIP = 3           /* a HIP launch failed; see bcnf_last_hip_error */
};

/* Mirrors CondRealNVP_v2.__init__ kwargs (cnf.py:358-375) for the coupling stack. */
typedef struct BcnfStackDesc {
  int32_t size;                      /* D                                     */
  int32_t n_conditions;              /* C (features per sample, h.shape[1])   */
  int32_t n_hidden;                  /* len(nested_sizes)                      */
  int32_t hidden[BCNF_MAX_HIDDEN];   /* nested_sizes                           */
  int32_t n_blocks;                  /* n_blocks                               */
  int32_t act_norm;                  /* 0/1                                    */
  int32_t two_way;                   /* 0/1 (the fused family requires 0)      */
  float dropout;                     /* p of every nn.Dropout in the nested MLP */
} BcnfStackDesc;

/* 1 if this descriptor runs on the fused small-width kernel family, else 0. */
int bcnf_stack_supported(const BcnfStackDesc* desc);

/* Canonical flat layouts (state_dict order of layers.*, frozen orthonormal matrices excluded /
 * separate): n_trainable = #floats of ActNorm + coupling params, n_frozen = (n_blocks-1)*D*D. */
int bcnf_param_count(const BcnfStackDesc* desc, int64_t* n_trainable, int64_t* n_frozen);

/* Bytes of the packed-parameter buffer written by bcnf_pack_params. */
int bcnf_packed_bytes(const BcnfStackDesc* desc, int64_t* bytes);

/* Bytes of the forward->backward workspace (saved block inputs + dropout masks) for a batch. */
int bcnf_workspace_bytes(const BcnfStackDesc* desc, int64_t batch, int32_t training, int64_t* bytes);

/* Bytes of the per-workgroup gradient slab used by bcnf_stack_backward for a batch. */
int bcnf_slab_bytes(const BcnfStackDesc* desc, int64_t batch, int64_t* bytes);

/* Re-lay params (canonical flat, n_trainable floats) and qmats ((n_blocks-1)*D*D floats) into
 * `packed` (bcnf_packed_bytes). Also writes the ActNorm log|det| constant used by the forward. */
int bcnf_pack_params(const BcnfStackDesc* desc, const float* params, const float* qmats, void* packed,
                     void* stream);

/* Forward of the whole stack given features h (B x C): z (B x D), ldj (B), optional log_prob (B).
 * training != 0 applies dropout with the counter-based RNG keyed by rng_state[0] (seed) and
 * rng_state[1] (offset), both read from DEVICE memory (graph-replay safe).
 * workspace != NULL saves what bcnf_stack_backward needs (bcnf_workspace_bytes). */
int bcnf_stack_forward(const BcnfStackDesc* desc, const void* packed, const float* y, const float* h,
                       int64_t batch, float* z, float* ldj, float* log_prob, int32_t training,
                       const uint64_t* rng_state, void* workspace, void* stream);

/* Backward: given dz (B x D) and dldj (B) (either may be NULL = zeros), writes dh (B x C,
 * overwritten, nullable), dy (B x D, nullable) and the per-workgroup gradient slabs into `slab`
 * (bcnf_slab_bytes). With dparams != NULL it then reduces the slabs into dparams (canonical flat,
 * n_trainable floats, overwritten); with dparams == NULL the caller runs bcnf_grad_reduce.
 * `training` and `workspace` must be those of the forward call. */
int bcnf_stack_backward(const BcnfStackDesc* desc, const void* packed, const float* h, const float* dz,
                        const float* dldj, int64_t batch, int32_t training, const void* workspace, float* dy,
                        float* dh, float* dparams, void* slab, void* stream);

/* Deterministic (fixed-order) sum of the slabs of a backward over `batch` samples into dparams.
 * Replaces autograd's implicit batch reduction of the parameter gradients. */
int bcnf_grad_reduce(const BcnfStackDesc* desc, const void* slab, int64_t batch, float* dparams, void* stream);

/* Inverse of the whole stack: y (N x D) from z (N x D). Row r uses feature row
 * cond_index[r] of h when cond_index != NULL (h then has any number of rows), else row r. */
int bcnf_stack_inverse(const BcnfStackDesc* desc, const void* packed, const float* z, const float* h,
                       const int64_t* cond_index, int64_t n_rows, float* y, int32_t training,
                       const uint64_t* rng_state, void* stream);

const char* bcnf_status_string(int status);
int bcnf_last_hip_error(void);

#ifdef __cplusplus
}
#endif

#endif /* BCNF_AMD_H */
