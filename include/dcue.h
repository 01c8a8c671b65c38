/*
 * dcue.h -- C ABI of libdcue_hip.so, the MI355X (gfx950) DCUE training-step library.
 *
 * The reference (estebandito22/Amplifai-DeepContentRecommenders) is pure Python/PyTorch; its
 * "operator interface" for the hot path is the torch module/trainer API listed per entry point
 * below. These entry points are what a ctypes binding of that interface calls.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer unless the name ends in _host. The caller (PyTorch's caching
 *    allocator in the shipped binding) owns every buffer; the library allocates nothing.
 *  - Every call is asynchronous on `stream` (a hipStream_t passed as void*) and returns a
 *    dcue_status; argument errors are detected on the host before anything is launched.
 *  - Float math is fp32 throughout (f32-input MFMA, exact f32 products); spectrogram tables may be
 *    stored as fp16 (lossless for fp16-representable inputs) or fp32.
 *  - Layouts: spectrogram table [n_tracks][n_frames=131][n_mels=128] (frame-major rows of mel bins);
 *    dense parameters are ONE flat fp32 buffer in reference parameter order and reference tensor
 *    layouts (offsets from dcue_param_layout); the user-embedding table is a separate
 *    [n_users][user_embdim] buffer (sharded by user across ranks).
 */
#ifndef DCUE_H_
#define DCUE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCUE_ABI_VERSION 16
#define DCUE_N_MELS 128
#define DCUE_N_FRAMES 131
#define DCUE_N_BN 6
/* dense parameter segments, reference order (DCUENet.named_parameters(), minus the embeddings):
 * 28 of the reference's DCUENet, then the text tower's text.conv.{weight, bias} (empty in the
 * audio-only towers) */
#define DCUE_N_DENSE_SEGMENTS 30

typedef enum {
  DCUE_OK = 0,
  DCUE_ERR_INVALID = 1,     /* bad argument (null pointer, size out of range) */
  DCUE_ERR_UNSUPPORTED = 2, /* valid for the reference, not for this build (e.g. d > 256) */
  DCUE_ERR_HIP = 3,         /* a HIP launch failed */
  DCUE_ERR_WORKSPACE = 4    /* workspace too small */
} dcue_status;

/* Item towers DCUENet wires by model_type (dcue/dcue.py:49-59):
 *   BN    truedcuemel1dbn    bn0 -> 4x[conv, pool, relu, bn] -> conv, relu, bn -> fc(d -> d) (default)
 *   PLAIN truedcuemel1d      the same without any BatchNorm
 *   RES   truedcuemel1dres   no BN; each block's output also time-averaged (AvgPool1d over all its
 *                            positions) and concatenated with the last block: fc(4H + d -> d)
 *   RESBN truedcuemel1dresbn RES with the BN tower's BatchNorms (the averages taken after each BN)
 * In the towers without BN the segments of the BN parameters are empty (dcue_param_layout).
 *   TEXT  BASELINE config 4, the mixed audio + text item encoder (no reference code: the reference's
 *         text item set, datasets/dcuelmitemset.py:8, imports a WordEmbeddings module it never
 *         published; this build's encoder): the BN tower's audio stack plus a text
 *         branch over each track's sentence of token ids (BOS + sentence + EOS, PAD-padded to
 *         text_len, dcuelmitemset.py:40-56): frozen word vectors [n_words][word_dim] (the
 *         LM-pretrained part, caller supplied: dcue_model.words), Conv1d(word_dim -> text_dim, k 3,
 *         pad 1), max over the non-PAD positions, ReLU; f = fc([s ; bn5(y5)]) with fc(text_dim + d -> d).
 *         The text positions' token ids come from dcue_tracks.tokens. */
#define DCUE_TOWER_BN 0
#define DCUE_TOWER_PLAIN 1
#define DCUE_TOWER_RES 2
#define DCUE_TOWER_RESBN 3
#define DCUE_TOWER_TEXT 4

typedef struct dcue_dims {
  int32_t conv_hidden; /* H: nn/dcue.py:45 conv_hidden (1..256; stored padded, dcue_storage_dims) */
  int32_t feature_dim; /* d: feature_dim (1..256; the trainer's default is 100, nn/dcue.py:44) */
  int32_t user_embdim; /* E: u_embdim (<= 1024) */
  int32_t tower;       /* DCUE_TOWER_* */
  int64_t n_users;     /* rows of the (local shard of the) user table */
  /* DCUE_TOWER_TEXT only (0 otherwise): */
  int32_t text_dim;    /* C: text features (1..256; stored at 64/128/256 channels) */
  int32_t word_dim;    /* E_w: word-vector width (4..1024, a multiple of 4) */
  int32_t text_len;    /* T: token positions per track (max_sentence_length + 1; 2..128) */
  int32_t text_pad;    /* PAD token id: positions holding it are left out of the max */
} dcue_dims;

/* Deferred user-table Adam (optional, selected by dcue_model.emb_step != NULL).
 * The reference's dense embedding gradient makes torch.optim.Adam step EVERY user row each batch,
 * with g = 0 (+ wd*p) for rows outside the batch (nn/dcue.py:143-147,209). Deferred mode performs
 * exactly those steps, later: a row's zero-gradient steps are replayed with the same fp32
 * operations and the same per-step scalars (kept in this log's history ring) right before the row
 * is next read (dcue_forward / dcue_user_tower bring their users' rows current), for a rolling
 * 1/cap slice of the table every step (so every row at least once per `cap` steps), and for all
 * rows on dcue_embedding_flush. After a flush the table and both moments are
 * bit-identical to the dense sweep's; between flushes rows outside recent batches lag behind, so
 * read the table directly only after a flush. The [cap][8] float history follows this header. */
typedef struct dcue_emb_log {
  int32_t step_done;   /* last Adam step recorded */
  int32_t flush_step;  /* every row is current to at least this step */
  int32_t n_touched;   /* emb_rows entries written by the last backward */
  int32_t grad_step;   /* the Adam step the last backward's compact gradient belongs to */
  int32_t cap;         /* history ring capacity in steps (= flush period) */
  /* frozen rows (ABI 16): the epoch whose steps all keep long-idle rows long idle -- its first step
   * (0: none), the largest |lr / bias_correction1| and the smallest eps it admits; a row's clock
   * (emb_step) with bit 30 set is frozen under it. Written by the library only. */
  int32_t frz_start;
  float frz_S;
  float frz_eps;
} dcue_emb_log;

/* Model state. Replaces DCUENet's parameters/buffers (dcue/dcue.py:21-68) + torch.optim.Adam state. */
typedef struct dcue_model {
  dcue_dims dims;
  float* params;       /* flat dense params, dcue_param_layout offsets */
  float* grads;        /* same layout */
  float* exp_avg;      /* Adam first moment, same layout */
  float* exp_avg_sq;   /* Adam second moment, same layout */
  float* emb;          /* [n_users][E] user_embd.embeddings.weight */
  float* emb_exp_avg;
  float* emb_exp_avg_sq;
  float* emb_grad;     /* [max_rows][E] compact rows of the embedding gradient (one per distinct user) */
  int32_t* emb_slot;   /* [n_users] slot of each user row in emb_grad, -1 = no gradient this step */
  float* bn_stats;     /* running_mean/var per BN layer, dcue_bn_layout offsets */
  int64_t* bn_batches; /* [6] num_batches_tracked */
  float* wpack;        /* packed conv weights (dcue_wpack_floats), refreshed by dcue_pack_weights */
  int64_t* emb_rows;   /* [max_rows] user row of each compact gradient row (-1: duplicate user) */
  int32_t* emb_step;   /* deferred mode: [n_users] step each row is current to (NULL: dense sweep) */
  dcue_emb_log* emb_log; /* deferred mode: header + history (dcue_emb_log_bytes) */
  int32_t emb_log_cap;   /* deferred mode: the log's history capacity (1..DCUE_MAX_LOG_CAP) */
  int32_t reserved;
  /* DCUE_TOWER_TEXT: the frozen word vectors text.embeddings.weight [n_words][word_dim] (never
   * updated by the library) and the power of two 2^words_exp the kernels scale them by before their
   * fp16 hi/lo split (exact; choose it so max |word value| * 2^words_exp lies in [2^13, 2^15)) */
  const float* words;
  int64_t n_words;
  int32_t words_exp;
  int32_t reserved2;
} dcue_model;

#define DCUE_MAX_LOG_CAP 256

/* One training batch, already resident in HBM.
 * Items are the spectrograms the item tower runs on. Catalogue mode (datasets/dcuedataset.py:242-250):
 * M = B*(1+N) items, item b = positive of row b, item B+b*N+j = negative j of row b. In-batch mode
 * (nn/dcue.py:698-709): M = B, negative (b,j) is a copy of positive neg_item[b][j]; the library runs
 * the tower once per distinct item and weights BatchNorm statistics by each item's copy count, which
 * is exactly the reference's computation on the duplicated [pos; neg] stack. */
#define DCUE_LAYOUT_CATALOGUE 0 /* M = B*(1+N), item b = positive b, item B+b*N+j = negative (b,j) */
#define DCUE_LAYOUT_GATHER 1    /* positives are items 0..B-1, negative (b,j) = item neg_item[b][j] */

typedef struct dcue_batch {
  int32_t n_rows;            /* B */
  int32_t n_neg;             /* N */
  int32_t n_items;           /* M */
  int32_t layout;            /* DCUE_LAYOUT_* */
  const int64_t* users;      /* [B] local user rows */
  const int32_t* item_track; /* [M] track row of each item */
  const int32_t* neg_item;   /* [B][N] item of each negative copy (GATHER layout; ignored otherwise) */
} dcue_batch;

typedef struct dcue_tracks {
  const void* data;  /* [n_tracks][131][128] */
  int64_t n_tracks;
  int32_t dtype;     /* 0 = fp16, 1 = fp32 */
  int32_t reserved;
  const int32_t* tokens;  /* DCUE_TOWER_TEXT: [n_tracks][text_len] token ids (< n_words) */
} dcue_tracks;

#define DCUE_ADAM_DENSE 1     /* flat dense params, then the conv-weight repack */
#define DCUE_ADAM_EMBEDDING 2 /* the user table */

typedef struct dcue_adam_args {
  /* param_group values set by CyclicLRWithRestarts, as the Python floats torch.optim.Adam reads
   * (double: 1 - beta1 etc. are formed in double and rounded once, as torch does) */
  double lr, beta1, beta2, eps, weight_decay;
  int32_t step;                              /* Adam step count AFTER increment (1 on first step) */
  int32_t parts;                             /* DCUE_ADAM_* mask; 0 = both */
  double grad_div; /* > 1: the dense gradient is first divided by it in place (DDP's mean over
                      grad_div ranks of an all-reduced sum); 0 or 1: used as is */
} dcue_adam_args;

/* ---------------------------------------------------------------------------------- layout */
int dcue_abi_version(void);
/* The HIP call behind the most recent DCUE_ERR_HIP (file:line, call, HIP error), "" if none. */
const char* dcue_last_error(void);
/* Kernel launches the library has issued in this process (all threads and streams; a step replay
 * through a captured graph counts none). Diagnostic: bench.py reports launches per step from it. */
int64_t dcue_launch_count(void);
/* Storage widths. Any conv_hidden / feature_dim in 1..256 is accepted (DCUENet takes any,
 * dcue/dcue.py:39-47). The library stores and computes them at the width rounded up to 32, 64, 128
 * or 256: every dense segment below is laid out for the storage dims (e.g. conv.layer5.weight is
 * [d_s][H_s][1], conv.fc.weight [d_s][d_s], or [d_s][4H + d_s] in the res towers, whose four
 * time-pooled blocks keep H columns each), and the reference-shaped parameter is the leading
 * [:d, :H, ...] corner of its segment. The caller zero-fills everything outside those corners
 * (weights, biases, BN gamma/beta and running statistics); the padded channels then carry exact
 * zeros through forward, backward and every optimizer, so they never leave zero and the corners
 * compute the reference model. Item / user feature outputs are [.][d_s] rows, zero past d. */
int dcue_storage_dims(const dcue_dims* dims, dcue_dims* storage_host);
/* offsets[DCUE_N_DENSE_SEGMENTS+1] (floats) of each dense parameter in `params` (storage dims) */
int dcue_param_layout(const dcue_dims* dims, int64_t* offsets_host);
/* offsets[2*DCUE_N_BN+1]: running_mean(l), running_var(l) for l = 0..5 */
int dcue_bn_layout(const dcue_dims* dims, int64_t* offsets_host);
int dcue_wpack_floats(const dcue_dims* dims, int64_t* n_floats_host);
int dcue_workspace_bytes(const dcue_dims* dims, int32_t max_rows, int32_t max_neg,
                         int32_t max_items, size_t* bytes_host);
/* Byte offsets inside a workspace carved for (B, N, M) of the forward outputs a train/eval
 * dcue_forward leaves there: [0] scores [B][N], [1] user feats [B][d_s], [2] item feats [M][d_s],
 * [3] loss (one float). Valid until the next call on the same workspace. */
int dcue_workspace_outputs(const dcue_dims* dims, int32_t B, int32_t N, int32_t M,
                           size_t* offsets_host);
/* Inspection (tests): byte offsets of the train forward's per-layer activations in the same
 * workspace. offsets[2(l-1)] = y_l, float [M][Lp_l][C_l] = relu(max-pooled conv + bias), before
 * BN; offsets[2(l-1)+1] = its uint8 [M][Lp_l][C_l] window argmax (0..pool-1, first maximum), for
 * conv layers l = 1..5 (Lp = 33, 8, 2, 1, 1; C = H_s, H_s, H_s, H_s, d_s: storage widths). */
int dcue_workspace_activations(const dcue_dims* dims, int32_t B, int32_t N, int32_t M,
                               size_t* offsets_host);

/* ------------------------------------------------------------------------- hot-path entries */
/* Refresh wpack from params (after any host-side write of conv weights and after every Adam step). */
int dcue_pack_weights(const dcue_model* m, void* stream);

/* Forward: DCUENet.forward(u, pos, neg) (dcue/dcue.py:70-108) + hinge loss (nn/dcue.py:167-170).
 * train != 0: model.train() semantics -- BatchNorm batch statistics over all copies, running stats
 * and num_batches_tracked updated, activations kept in `ws` for dcue_train_backward.
 * train == 0: model.eval() semantics (running statistics, nothing updated).
 * Outputs (each nullable): scores[B][N], user feats [B][d_s], item feats [M][d_s], loss[1] (mean over
 * rows of the summed hinge). */
int dcue_forward(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws,
                 size_t ws_bytes, int32_t train, float margin, float* scores, float* user_feat,
                 float* item_feat, float* loss, void* stream);

/* Backward of the last train-mode dcue_forward on the same ws: loss.backward() (nn/dcue.py:208).
 * dscores == NULL: gradient of the hinge loss; else dL/dscores [B][N] from the caller.
 * Writes m->grads (dense, overwritten) and the compact embedding gradient (emb_grad/emb_slot),
 * scaled by emb_grad_scale (1/world_size under user-sharded data parallelism). */
int dcue_train_backward(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws,
                        size_t ws_bytes, const float* dscores, float emb_grad_scale, void* stream);

/* ------------------------------------------------------------ DCBR path (BASELINE config 5)
 * The reference never published it (dcrecommend/dcbr is git-ignored, .gitignore:13;
 * nn/dcue_orig.py:35 imports it and fails), so these restate the papers and are parity-unpinned
 * against the reference (pinned against oracle/wrmf_oracle.py and the fp64 oracle item tower).
 *
 * WRMF (Hu, Koren, Volinsky 2008) half-step: every row r of `solve` [n_rows][dim] becomes
 *   x_r = (F^T F + sum_{j in r} (c_rj - 1) f_j f_j^T + lambda I)^{-1} sum_{j in r} c_rj f_j,
 *   c_rj = 1 + alpha * v_rj (v = values, or 1 when values == NULL),
 * with F = `fixed` [n_fixed][dim] and row r's observed columns indices[indptr[r] .. indptr[r+1]).
 * Rows without an observed column get x_r = 0. dim <= 128; lambda > 0. Alternate users and items
 * (the item-side CSR is the transpose) for the ALS iterations. fp64 throughout: rows with at most
 * 32 observed columns through the Woodbury identity over (F^T F + lambda I)^{-1}, the others by a
 * block Cholesky (fp64 MFMA). The workspace holds the Gram partials, G, and that inverse. */
int dcue_wrmf_workspace_bytes(int32_t dim, int64_t n_fixed, size_t* bytes_host);
int dcue_wrmf_half_step(float* solve, int64_t n_rows, const float* fixed, int64_t n_fixed, int32_t dim,
                        const int64_t* indptr, const int32_t* indices, const float* values, float alpha,
                        float lambda, void* ws, size_t ws_bytes, void* stream);
/* DCBR regression step (van den Oord, Dieleman, Schrauwen 2013): the item tower's train forward over
 * the batch's items (catalogue layout, n_neg = 0, n_rows = n_items = M; users unused), the MSE loss
 * mean over [M][d] of (f - target)^2 (torch.nn.MSELoss; target [M][d_s] rows, columns past d
 * ignored) into *loss (device, nullable), and its backward into the item tower's gradients in
 * m->grads (the user-tower segments are left as they are). Workspace: dcue_workspace_bytes(dims, M,
 * 0, M). BN running statistics update as in dcue_forward. */
int dcue_dcbr_step(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, const float* target,
                   float* loss, void* ws, size_t ws_bytes, void* stream);

/* optimizer.step() (nn/dcue.py:209, torch.optim.Adam semantics): dense params + every user row
 * (rows without a gradient this step still decay their moments and move, as the reference's dense
 * embedding gradient does), then clears emb_slot and refreshes wpack. In deferred mode the user
 * table part steps the batch's rows now and records the step for the others (dcue_emb_log); steps
 * must then be consecutive (a->step == step_done + 1). */
int dcue_adam_step(const dcue_model* m, const dcue_adam_args* a, void* stream);

/* The trainer's other optimizers, DCUE(optimize='sgd' | 'ranger') (nn/dcue.py:148-157): one step
 * over the dense flat buffer and every user-table row (the dense embedding gradient: rows outside
 * the batch step with g = 0), then the conv-weight repack. Per-element arithmetic as torch's CPU
 * kernels round it (oracle/optim_oracle.py), sqrt correctly rounded. */
#define DCUE_OPT_SGD 1    /* torch.optim.SGD(lr, momentum=beta1, weight_decay, nesterov=True) */
#define DCUE_OPT_RANGER 2 /* optim/ranger.py:26-165: RAdam + Lookahead */
typedef struct dcue_opt_args {
  int32_t kind;           /* DCUE_OPT_* */
  int32_t step;           /* step count after increment (1 on the first step) */
  double lr, beta1, beta2, eps, weight_decay; /* SGD: beta1 = momentum; beta2, eps unused */
  double alpha;           /* Ranger: lookahead interpolation (0.5 in the trainer) */
  int32_t k;              /* Ranger: lookahead period (6) */
  int32_t reserved;
  double n_sma_threshold; /* Ranger: RAdam rectification threshold (5) */
  double grad_div;        /* as dcue_adam_args.grad_div */
} dcue_opt_args;
/* Optimizer state, caller-owned, zero-initialised before the first step except the lookahead
 * buffers, which start as copies of the parameters (optim/ranger.py:113-114).
 *   SGD: a = momentum buffer.   Ranger: a = exp_avg, b = exp_avg_sq, c = slow (lookahead) weights.
 * dense_*: [n_dense] like params; emb_*: [n_users][E] like the user table. */
typedef struct dcue_opt_state {
  float *dense_a, *dense_b, *dense_c;
  float *emb_a, *emb_b, *emb_c;
} dcue_opt_state;
int dcue_optimizer_step(const dcue_model* m, const dcue_opt_args* a, const dcue_opt_state* st, void* stream);

/* Deferred user-table Adam: log size for a `cap`-step history; (re)initialise the log and row
 * clocks at Adam step `step` (table and moments current to it); bring `users`' rows current;
 * bring every row current (the state then equals the dense sweep's bit for bit). */
int dcue_emb_log_bytes(int32_t cap, size_t* bytes_host);
int dcue_emb_log_init(const dcue_model* m, int32_t cap, int32_t step, void* stream);
int dcue_embedding_sync(const dcue_model* m, const int64_t* users, int32_t n, void* stream);
int dcue_embedding_flush(const dcue_model* m, void* stream);

/* Eval-mode item tower (running BN stats): DCUENet.conv(X) under model.eval() (nn/dcue.py:663).
 * item_feat: [n_items][d_s]. */
int dcue_item_tower_eval(const dcue_model* m, const dcue_tracks* t, const int32_t* item_track,
                         int32_t n_items, void* ws, size_t ws_bytes, float* item_feat, void* stream);
/* Eval user tower: DCUENet.user_embd(idx) (nn/dcue.py:638). user_feat: [n][d_s]. */
int dcue_user_tower(const dcue_model* m, const int64_t* users, int32_t n, void* ws, size_t ws_bytes,
                    float* user_feat, void* stream);

/* Layout conversion of caller-provided spectrograms: [M][128][131] (the reference's per-track tensor,
 * datasets/dcuedataset.py:234-235) -> [M][131][128] track rows (the table layout). */
int dcue_transpose_spectrograms(const float* ncl, int32_t M, float* out, void* stream);
/* Catalogue batch assembly (datasets/dcuedataset.py:242-250 + dcue/dcue.py:90 concat order):
 * item_track = [pos_items[0..B); neg_items[b][j] at B + b*N + j]. */
int dcue_build_catalogue_batch(const int64_t* pos_items, const int64_t* neg_items, int32_t B,
                               int32_t N, int32_t* item_track, void* stream);

/* ------------------------------------------------------------------------------ samplers */
/* MT19937 state (numpy legacy RandomState): 624 words + position, in device memory. */
typedef struct dcue_mt_state {
  uint32_t key[624];
  int32_t pos;
  int32_t pad[3];
} dcue_mt_state;

/* np.random.seed(seed) into a device state (init_genrand). */
int dcue_mt_seed(dcue_mt_state* state, uint32_t seed, void* stream);
/* n tempered 32-bit outputs, advancing the state (genrand_int32). */
int dcue_mt_draw(dcue_mt_state* state, uint32_t* out, int32_t n, void* stream);
/* In-batch negatives (nn/dcue.py:698-709): neg[b][j] = masked draw over the B-1 other rows, from
 * one global stream, row-major. Bit-exact with numpy for the same state. */
int dcue_sample_inbatch(dcue_mt_state* state, int32_t B, int32_t N, int32_t* neg, void* stream);
/* Catalogue negatives (datasets/dcuedataset.py:207-220): for each sample the user's non-items in
 * the split (split_items sorted; user_split_rank = CSR over users of the ranks, inside split_items,
 * of the user's split items, sorted), N draws with replacement. reseed != 0: every sample draws from
 * a fresh stream seeded with `seed` (random_seed mode); else all samples share `state` in order.
 * Writes item ids (values of split_items). A user with no non-item in the split (numpy raises
 * ValueError there) gets a row of -1 and consumes no draw: callers check for such users on the host
 * (their CSR row length >= n_split) and raise before sampling them; dcue_build_catalogue_batch
 * maps a -1 to item 0 so it never reads outside the track table. */
int dcue_sample_catalogue(dcue_mt_state* state, int32_t reseed, uint32_t seed,
                          const int64_t* split_items, int64_t n_split, const int64_t* user_indptr,
                          const int32_t* user_split_rank, const int64_t* users, int32_t n_samples,
                          int32_t N, int64_t* out, void* stream);

/* -------------------------------------------------------------------------- step plans */
/* A training-step plan: the step's kernels (optionally the in-batch negative draw, then the train
 * forward and backward of dcue_forward/dcue_train_backward) bound once and issued by one host call
 * per step. The model, batch, tracks and workspace buffers are bound at creation (their addresses
 * must stay valid and unchanged); their CONTENTS are read at each launch, so the caller refreshes
 * the batch buffers between launches (or passes sources to dcue_plan_launch, which copies them in
 * stream order first). The optimizer step stays outside (its scalars change every step), as does
 * any gradient all-reduce between the two. Replay is eager (issued from C++ onto the caller's
 * stream + side streams) unless DCUE_PLAN_GRAPH asks for a captured HIP graph. */
typedef struct dcue_plan dcue_plan;
#define DCUE_PLAN_SAMPLE_INBATCH 1 /* step starts with dcue_sample_inbatch(mt, B, N, b->neg_item) */
#define DCUE_PLAN_GRAPH 2          /* capture into a HIP graph and replay that */
typedef struct dcue_plan_config {
  int32_t flags;        /* DCUE_PLAN_* */
  float margin;         /* hinge margin (nn/dcue.py:167-170) */
  float emb_grad_scale; /* as dcue_train_backward */
  int32_t reserved;
  dcue_mt_state* mt;    /* sampler state (DCUE_PLAN_SAMPLE_INBATCH) */
} dcue_plan_config;
int dcue_plan_create(const dcue_model* m, const dcue_batch* b, const dcue_tracks* t, void* ws,
                     size_t ws_bytes, const dcue_plan_config* cfg, dcue_plan** plan_host);
/* users_src / item_track_src (nullable): copied into the bound batch buffers before the replay. */
int dcue_plan_launch(dcue_plan* plan, const int64_t* users_src, const int32_t* item_track_src,
                     void* stream);
/* dcue_plan_launch, then (adam != NULL) dcue_adam_step on the plan's model: one host call per
 * training step (a bound communicator's exchange included, dcue_plan_set_comm). Without a
 * communicator the dense Adam is split: bn0 / conv 1 / bn1 on `stream` right behind the conv-1
 * weight gradient, the other segments on the library's user stream once the side streams'
 * gradients are in, so `stream` never waits for that join; the plan's next launch waits for it
 * before conv 2. Until then the parameters are current only for work ordered after dcue_plan_sync
 * (every library entry point that reads them joins by itself). */
int dcue_plan_step(dcue_plan* plan, const int64_t* users_src, const int32_t* item_track_src,
                   const dcue_adam_args* adam, void* stream);
/* `stream` waits for everything the plan's last step left on the library's side streams. */
int dcue_plan_sync(dcue_plan* plan, void* stream);
/* Data-parallel overlap (row e): `stream` waits until every side-stream part of the plan's last
 * launched step is in. From then on the flat gradient buffer is final except its first
 * DCUE_SEG_LATE segments (bn0, conv layer 1, bn1: written by the caller's stream at the step's end),
 * so an all-reduce of the rest issued on `stream` overlaps the conv-1 weight gradient. Eager plans
 * only (DCUE_ERR_INVALID for a graph plan or before the first launch). Replaces the single
 * post-backward all-reduce of the DDP-style loop (nn/dcue.py:208-209 under data parallelism). */
#define DCUE_SEG_LATE 6
int dcue_plan_wait_side(dcue_plan* plan, void* stream);
/* Lookahead (eager plans of a BatchNorm tower): announces the item_track_src buffer of the
 * NEXT launch ([M] int32 device ids, contents fixed until that launch). The following launch then
 * also prepares that batch's model-independent item inputs beside its own step -- bn0's batch
 * statistics (k_input_stats) and bn0(x) zero-padded for the conv-1 weight gradient (k_xhat0) -- so
 * the next step's chain starts at conv 1. A next launch whose item_track_src is not the announced
 * buffer computes them itself, as without lookahead; NULL withdraws the announcement. The batch
 * composition of the reference is likewise prepared ahead, by its DataLoader workers
 * (nn/dcue.py:711-721). The announced items must be written, in `stream` order, before the
 * announcing launch (the lookahead reads them after that launch's score kernel, on a side stream).
 * DCUE_ERR_UNSUPPORTED for graph or BatchNorm-free plans. */
int dcue_plan_set_next(dcue_plan* plan, const int32_t* next_item_track);

/* ---- check mode (a HIP bounds/NaN check mode; the reference has none) ----
 * Probes run between steps. Each ORs `bit` into the device word *flags when it finds a problem and
 * never faults on the data it inspects: ids can be validated before a step indexes with them, and
 * the loss, parameters, gradients and user table after it. */
int dcue_check_finite(const float* buf, int64_t n, int32_t* flags, int32_t bit, void* stream);
/* ids: int32 (id_bytes 4) or int64 (8); flags any id outside [0, limit). */
int dcue_check_ids(const void* ids, int32_t id_bytes, int64_t n, int64_t limit, int32_t* flags, int32_t bit,
                   void* stream);
int dcue_plan_destroy(dcue_plan* plan);

/* ---- debug: schedule perturbation, probes, poison (no reference counterpart) ----
 * dcue_debug_delay: every later step launches, ahead of the work at `site`, a spin kernel of
 * `microseconds` (0: none, at most 1e6) on that work's stream. A step's results are bit-identical
 * under any delays -- every buffer is ordered by the streams' events, not by timing -- so a
 * difference names a missing cross-stream wait (tests/test_gpu_races.py). */
#define DCUE_SITE_USER_FWD 0   /* user stream: the user tower's forward (deferred-row sync + GEMMs) */
#define DCUE_SITE_USER_BWD 1   /* user stream: the user tower's backward + user-table Adam */
#define DCUE_SITE_WGRAD_HI 2   /* wgrad stream 0: weight gradients of conv layers 3-5 (+ fc) */
#define DCUE_SITE_WGRAD_2 3    /* wgrad stream 1: weight gradient of conv layer 2 */
#define DCUE_SITE_FC_WGRAD 4   /* wgrad stream 1: res / text towers' fc (+ text conv) weight gradients */
#define DCUE_SITE_LATE_ADAM 5  /* split plans: the late segments' Adam (user or comm stream) */
#define DCUE_SITE_PROLOGUE 6   /* plans: the next step's prologue (wgrad stream 0) */
#define DCUE_SITE_LOOKAHEAD 7  /* plans: the announced next batch's input statistics (wgrad stream 0) */
#define DCUE_SITE_CONV2 8      /* caller's stream: conv 2 forward */
#define DCUE_SITE_DGRAD_2 9    /* caller's stream: conv-2 input gradient (g1) */
#define DCUE_SITE_WGRAD_1 10   /* caller's stream: conv-1 weight gradient */
#define DCUE_SITE_TEXT_FWD 11  /* text tower: the text branch's forward on its side stream (ABI 16) */
#define DCUE_N_DEBUG_SITES 12
int dcue_debug_delay(int32_t site, int32_t microseconds);
/* Probes: buf = NULL (off) or a device array of dcue_debug_probe_count() records
 * { uint32 nonfinite; uint32 nonzero; uint64 first_bad } (the caller sets first_bad to UINT64_MAX
 * and the rest to 0). While bound, steps check the output of each probed launch on its own stream
 * (no added cross-stream order): a non-finite element sets `nonfinite` and takes the minimum of the
 * device's 100 MHz wall clock into `first_bad`; any non-zero element sets `nonzero`. The record with
 * the smallest first_bad names the first launch that wrote a non-finite value. */
int dcue_debug_probes(void* buf);
int dcue_debug_probe_count(void);
const char* dcue_debug_probe_name(int32_t i);
/* on != 0: plans created afterwards fill the scratch they allocate with 0xFF bytes (float NaN). */
int dcue_debug_poison(int32_t on);
/* Reads and clears the current device's word that the fused user-tower forward sets when a bounded
 * wait for another workgroup's row gave up (bit 0; never expected). bench.py fails its line on a
 * non-zero value. */
int dcue_debug_fail_flags(uint32_t* flags_host);
/* ORs `bits` into the current device's fail word (tests: a forced flag must fail the bench line; ABI 16). */
int dcue_debug_raise_fail_flags(uint32_t bits);

/* ------------------------------------------------- data-parallel gradient exchange (RCCL) */
/* One process per GPU; users are sharded over the ranks, so the only exchange of a step is the
 * mean over ranks of the replicated dense gradient (the flat buffer, dcue_param_layout). The
 * library drives RCCL itself so that a data-parallel step stays one host call (dcue_plan_step).
 * The caller ships the unique id from rank 0 to the others (e.g. over torch.distributed). */
typedef struct dcue_comm dcue_comm;
#define DCUE_COMM_ID_BYTES 128
int dcue_comm_unique_id(void* id_host); /* rank 0: DCUE_COMM_ID_BYTES bytes */
/* A communicator over `world` ranks on the current HIP device (collective: every rank calls it). */
int dcue_comm_create(const void* id_host, int32_t world, int32_t rank, dcue_comm** comm_host);
/* A communicator whose transport is the caller's: `fn(ctx, host_buf, n, dtype)` must replace the n
 * elements at host_buf (DCUE_COMM_F32: float, DCUE_COMM_U64: uint64, two's-complement wrap) by their
 * sum over the ranks and return 0. The library drains its stream and stages the buffer through pinned
 * host memory around each call, so a plan step blocks the host at every exchange point; it runs the
 * same exchange code (buckets, event order, Adam's divide) as the RCCL transport. For ranks that
 * cannot share an RCCL communicator -- several ranks on one GPU over gloo (tests) -- not for speed. */
#define DCUE_COMM_F32 0
#define DCUE_COMM_U64 1
typedef int (*dcue_host_allreduce_fn)(void* ctx, void* host_buf, int64_t n, int32_t dtype);
int dcue_comm_create_host(int32_t world, int32_t rank, dcue_host_allreduce_fn fn, void* ctx,
                          dcue_comm** comm_host);
int dcue_comm_destroy(dcue_comm* comm);
/* In-place mean over the ranks of n floats, ordered on `stream` (sum all-reduce, then / world). */
int dcue_comm_allreduce_mean(dcue_comm* comm, float* buf, int64_t n, void* stream);
/* In-place all-gather, ordered on `stream`: buf holds world * count floats, rank r's own part at
 * buf[r * count, (r + 1) * count); afterwards every rank holds every part (RCCL: ncclAllGather; the
 * host transport: the other parts zeroed, then the sum). The DCBR path's row-sharded WRMF half-steps
 * (each rank solves its rows, every rank needs all of them as the next half-step's fixed side). */
int dcue_comm_allgather(dcue_comm* comm, float* buf, int64_t count, void* stream);
/* Bind (or, with NULL, unbind) a communicator to an eager plan. dcue_plan_step then exchanges the
 * dense gradient between the backward and Adam, in two buckets on the communicator's stream: the
 * gradients the side streams finish (everything after DCUE_SEG_LATE) as soon as they are in,
 * overlapping the conv-1 weight gradient on the caller's stream, then bn0/conv-1/bn1 once the step
 * ends; Adam then divides by the world size (dcue_adam_args.grad_div) in its sweep. dcue_plan_launch
 * makes the same exchange and divides by the world size itself, so the gradient it leaves is the
 * mean over the ranks for any optimizer called after it (dcue_optimizer_step, dcue_adam_step with
 * grad_div 0). Collective order is the same on every rank. The plan must have been created with
 * emb_grad_scale = 1/world. */
int dcue_plan_set_comm(dcue_plan* plan, dcue_comm* comm);
/* SyncBN (on != 0; the bound communicator's ranks): every train-mode BatchNorm of the item
 * tower normalises over the whole global batch. Its exact fixed-point sums (forward: count-weighted
 * sum and sum of squares; backward: sum g and sum g*xhat) are all-reduced over the ranks between
 * their producer and first consumer, so the statistics -- and the running statistics -- are the same
 * on every rank and do not depend on the order of the ranks. BN gamma/beta gradients enter the
 * exchange as 1/world of the global sum each, so after the DDP mean they equal torch
 * SyncBatchNorm + DDP's (the mean of the per-rank local sums). 11 small collectives per step (6 BN
 * layers forward, bn5..bn1 backward; bn0 has no input gradient, its gamma/beta gradients stay local).
 * Requires a bound communicator (DCUE_ERR_INVALID otherwise) and the split-f16 weight gradients
 * (DCUE_ERR_UNSUPPORTED under DCUE_WGRAD_F16=0). Unbinding the communicator turns it off. */
int dcue_plan_set_sync_bn(dcue_plan* plan, int32_t on);

/* ------------------------------------------------------------------- live kernel timing */
/* enable = n > 0: every n-th launch of the kernel class (also inside plans created afterwards),
 * starting with the n-th after this call (ABI 16), gets a HIP event pair bound to the launch itself
 * (its dispatch's start and end); 0 disables.
 * dcue_timer_read waits for the recorded pairs, returns their summed time and count, and resets.
 * For bench rooflines: a timed launch costs the stream a few microseconds, so time a sample. */
#define DCUE_TIMED_CONV1_WGRAD 0 /* conv layer-1 weight gradient (the step's largest MFMA kernel) */
#define DCUE_TIMED_CONV1_FWD 1   /* conv layer-1 forward */
#define DCUE_TIMED_EMB_FLUSH 2   /* deferred user-table Adam: full-table flush */
#define DCUE_TIMED_ADAM_EMBED 3  /* dense user-table Adam sweep */
#define DCUE_TIMED_ALLREDUCE 4    /* a plan's RCCL gradient exchange (each bucket's all-reduce) */
#define DCUE_TIMED_EMB_SLICE 5    /* deferred user-table Adam: one step's rolling-flush slice */
#define DCUE_TIMED_TEXT_FWD 6     /* text tower: the text conv forward (k_text_fwd, config 4) */
#define DCUE_TIMED_USER_FWD 7     /* the fused user-tower forward (k_user_fwd; ABI 16) */
#define DCUE_TIMED_TEXT_WGRAD 8   /* text tower: the text conv's weight gradient (k_text_wgrad; ABI 16) */
#define DCUE_N_TIMED 9
int dcue_timer_enable(int32_t kernel, int32_t enable);
int dcue_timer_read(int32_t kernel, double* total_ms_host, int64_t* launches_host);
/* The same recorded launches one by one: each duration in ms into ms_host[0 .. min(n, cap)), the
 * count into *launches_host; resets (ABI 15). */
int dcue_timer_samples(int32_t kernel, float* ms_host, int64_t cap, int64_t* launches_host);

/* ------------------------------------------------------------------------ evaluation metrics */
/* Ranking metrics of DCUE's evaluation for a batch of queries (users for DCUE.score, songs for
 * DCUE.score_song), replacing the per-query predict() loops and sklearn calls of nn/dcue.py:380-476
 * and the candidate lists of datasets/dcuepredset.py:39-131.
 *   query_feat [n_query_rows][d], cand_feat [n_cand][d]: factors (DCUE.user_factors / item_factors,
 *     nn/dcue.py:629-668); scores are nn.CosineSimilarity(dim=1) of a query row and a candidate row.
 *   queries[n_queries]: query row of each evaluated query (a sample; repeats allowed, :413/:420).
 *   pos_ptr[n_query_rows+1], pos_idx: CSR over query rows of the candidates the query interacted
 *     with in ANY split (datasets/dcuedataset.py:74-89 item_user matrix), each row sorted, no repeats.
 *   cand_class[n_cand]: bit 0 = the candidate is in the pred list (the pred split's songs/users),
 *     bit 1 = in the truth list; 0 = in neither.
 *   DCUE_RANK_SPLIT (DCUE.score, :399-447): AUC weighted over {pred positives + truth negatives} and
 *     {pred negatives + truth positives}, AP over both; has_pos = the query has pred positives (the
 *     reference stops its user loop at the first query without, :393-394).
 *   DCUE_RANK_SINGLE (DCUE.score_song, :463-474): targets = 1 for the query's positives among the
 *     candidates with bit 1, 0 for EVERY candidate with bit 0 -- positives included: the reference's
 *     non-user list (dcuepredset.py:53-62) takes `getrow(i).nonzero()[0]`, the row indices (all 0),
 *     so it only drops user index 0 and keeps the song's own users as negatives too; callers set
 *     bit 0 on the split's users except user 0 and bit 1 on the split's users. AUC / AP over that
 *     list, 1/1 if every target is 1, 0/0 if none; has_pos = 0 marks a query the reference skips.
 *   has_pos bit 1: a score the reference would hand to sklearn is NaN or infinite -- there
 *     roc_auc_score / average_precision_score raise ValueError (:440, :447, :473-474), and the
 *     query's auc / ap here are meaningless (the binding raises ValueError instead of using them).
 * Exact tie-aware AUC (Mann-Whitney, ties 1/2) and step-wise AP from integer rank counts, fp64.
 * At most 4096 positives per query inside the lists (else DCUE_ERR_UNSUPPORTED). query_batch
 * queries are scored per pass; the workspace holds their [query_batch][n_cand] score rows.
 * Synchronises `stream` before returning. */
#define DCUE_RANK_SPLIT 0
#define DCUE_RANK_SINGLE 1
int dcue_rank_workspace_bytes(int64_t n_cand, int32_t d, int32_t query_batch, size_t* bytes_host);
int dcue_rank_metrics(const float* query_feat, int64_t n_query_rows, const float* cand_feat,
                      int64_t n_cand, int32_t d, const int32_t* queries, int32_t n_queries,
                      const int64_t* pos_ptr, const int32_t* pos_idx, const uint8_t* cand_class,
                      int32_t mode, int32_t query_batch, void* ws, size_t ws_bytes, double* auc,
                      double* ap, int32_t* has_pos, void* stream);
/* DCUE._item_factors' averaging (nn/dcue.py:655-668): f <- (f + f + ... n_iter times) / n_iter in
 * fp32, for 131-frame tracks whose n_iter eval passes are identical (no random crop). */
int dcue_factor_repeat_mean(float* f, int64_t n, int32_t n_iter, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DCUE_H_ */
