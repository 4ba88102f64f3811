/*
 * mcmc355.h — C-ABI of libmcmc355.so, the MI355X (gfx950) HMC / NUTS engine.
 *
 * This is the drop-in boundary for the reference's sampling hot path
 * (korentomas/mlx-mcmc):
 *
 *   reference symbol                                   replaced by
 *   -------------------------------------------------  ------------------------------
 *   mlx_mcmc/kernels/hmc.py:7-206   hmc()              mc_hmc_run (+ mc_state_init)
 *   mlx_mcmc/kernels/hmc.py:53-67   grad_log_prob      mc_logp_grad (tape evaluator)
 *   mlx_mcmc/kernels/hmc.py:69-100  leapfrog_step      (fused inside mc_hmc_run)
 *   mlx_mcmc/kernels/hmc.py:102-111 hamiltonian        (fused inside mc_hmc_run)
 *   mlx_mcmc/kernels/hmc.py:113-153 hmc_step           (fused inside mc_hmc_run)
 *   mlx_mcmc/kernels/nuts.py:16-358 nuts()             mc_nuts_run (+ mc_state_init)
 *   mlx_mcmc/kernels/metropolis.py:6-101               mc_mh_run (+ mc_state_init)
 *     metropolis_hastings()
 *   mlx_mcmc/kernels/nuts.py:137-218 build_tree        (iterative, inside mc_nuts_run)
 *   mlx_mcmc/kernels/nuts.py:119-135 no_u_turn         (inside mc_nuts_run)
 *   mlx_mcmc/distributions/normal.py:33-56 log_prob    MC_DIST_NORMAL term / mc_dist_log_prob
 *   mlx_mcmc/distributions/halfnormal.py:34-63         MC_DIST_HALFNORMAL term / mc_dist_log_prob
 *   mlx_mcmc/distributions/exponential.py:48-71        MC_DIST_EXPONENTIAL term / mc_dist_log_prob
 *   mlx_mcmc/distributions/gamma.py:40-88              MC_DIST_GAMMA term / mc_dist_log_prob
 *   mlx_mcmc/distributions/beta.py:37-91               MC_DIST_BETA term / mc_dist_log_prob
 *   mlx.core.random (key/split/normal/uniform)         Philox4x32-10 counter RNG, mc_rng_fill
 *   examples/06_nuts_comparison.py:22-41 compute_ess   mc_series_stats (MC_ST_ESS)
 *   README.md:214 roadmap "R-hat" (no reference code)  mc_stats_reduce + mc_rhat
 *   mlx_mcmc/inference/mcmc.py:191-227 summary         mc_pool_moments, mc_select
 *
 * The reference is pure Python on MLX and has no FFI of its own; the
 * Python host layer of this repository (mlx_mcmc_amd/_lib.py) binds these
 * symbols with ctypes — see INTEGRATION.md for the binding a maintainer of
 * the reference would add.
 *
 * Conventions
 *   - All array arguments named *_dev are device pointers (HIP, current
 *     device); the caller owns them.  The library owns only mc_program.
 *   - Every entry point returns 0 on success or a negative MC_ERR_* code;
 *     nothing throws or aborts across the ABI.  mc_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - Launch functions are asynchronous on the given stream and never
 *     allocate, free or synchronise (they are graph-capturable).
 *   - Parameters are one flat float32 vector of length n_params (the
 *     concatenation of the user's parameter dict in insertion order).
 */
#ifndef MCMC355_H
#define MCMC355_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2: mc_operand.transform (formerly `reserved`) and mc_term.affine are
 * read and validated (an unknown transform, or a transform on a non-parameter
 * operand, is MC_ERR_INVALID): callers written against ABI 1 must zero them. */
#define MC_ABI_VERSION 2

/* ---- error codes -------------------------------------------------------- */
#define MC_OK              0
#define MC_ERR_INVALID    -1   /* bad argument / malformed program           */
#define MC_ERR_UNSUPPORTED -2  /* well-formed but outside what the kernels do */
#define MC_ERR_HIP        -3   /* HIP runtime error                          */
#define MC_ERR_NOMEM      -4   /* device allocation failed                   */
#define MC_ERR_TIMEOUT    -5   /* a sliced launch's cross-workgroup exchange  */
                               /* did not complete (see mc_workspace_status)  */

/* ---- the tape: a log density as a sum of fused distribution terms ------- */
/* A term is  weight * sum_i dist(loc_i, scale_i).log_prob(value_i)  over n
 * broadcast elements.  This is exactly the shape every reference model takes
 * (e.g. tests/test_hmc.py:187-198, examples/02_hmc_comparison.py:40-52).   */
/* Operand slots of a term: value, then (loc | alpha), then (scale | rate |
 * beta).  The gammaln normalisers of Gamma and Beta are evaluated at the
 * current shape values but carry no gradient, exactly as the reference's
 * host-side scipy gammaln (gamma.py:48-59, beta.py:45-57).                   */
typedef enum {
    MC_DIST_NORMAL      = 0,  /* normal.py:33-56       (value, loc, scale)   */
    MC_DIST_HALFNORMAL  = 1,  /* halfnormal.py:34-63   (value, -, scale)     */
    MC_DIST_EXPONENTIAL = 2,  /* exponential.py:48-71  (value, -, rate)      */
    MC_DIST_GAMMA       = 3,  /* gamma.py:40-88        (value, alpha, beta)  */
    MC_DIST_BETA        = 4,  /* beta.py:37-91         (value, alpha, beta)  */
    MC_DIST_IDENTITY    = 5,  /* weight * sum_i value_i   (value, -, -):  a   */
                              /* parameter expression added to the log      */
                              /* density (the Jacobian of a reparameterised */
                              /* parameter, `lp + log_sigma`)               */
    MC_DIST_EXPR        = 6   /* weight * sum_i root_i of an elementwise     */
                              /* expression (mc_expr, mc_program_create_expr) */
} mc_dist_kind;

typedef enum {
    MC_OP_NONE    = 0,  /* operand unused (HalfNormal loc)                   */
    MC_OP_CONST   = 1,  /* broadcast float constant `value`                  */
    MC_OP_PSCALAR = 2,  /* broadcast parameter q[param_offset]               */
    MC_OP_DATA    = 3,  /* data[pool_offset + i]        (float32 data pool)  */
    MC_OP_PVEC    = 4,  /* q[param_offset + i]                               */
    MC_OP_GATHER  = 5   /* q[param_offset + index[pool_offset + i]] (int32)  */
} mc_operand_kind;

/* An elementwise transform of a parameter operand (PSCALAR / PVEC / GATHER),
 * applied in f32 before the term reads it, its derivative applied to the
 * operand's cotangent as mx.grad's VJPs do (exp: c * exp(x); log: c / x):
 * `Normal(mu, mx.exp(log_sigma))`, `Normal(0, 1).log_prob(mx.log(x))`.      */
typedef enum {
    MC_XF_NONE = 0,
    MC_XF_EXP  = 1,
    MC_XF_LOG  = 2
} mc_transform_kind;

typedef struct mc_operand {
    int32_t kind;          /* mc_operand_kind                               */
    int32_t param_offset;  /* PSCALAR / PVEC / GATHER                       */
    int64_t pool_offset;   /* DATA: float pool; GATHER: index pool          */
    float   value;         /* CONST                                         */
    int32_t transform;     /* mc_transform_kind (parameter operands only;   */
                           /* was `reserved`: zero-initialised callers get  */
                           /* MC_XF_NONE)                                   */
} mc_operand;

typedef struct mc_term {
    int32_t    dist;       /* mc_dist_kind                                  */
    int32_t    affine;     /* 0, or k + 1: the loc is affine, affines[k]    */
    int64_t    n;          /* broadcast length (>= 1)                       */
    float      weight;     /* multiplies the term (1.0 for `lp += term`)    */
    float      reserved1;
    mc_operand value, loc, scale;
} mc_term;

/* An affine loc (the reference differentiates any MLX expression of the
 * parameters, hmc.py:53-67; these are the linear-predictor forms):
 *     loc_i = loc_i + slope_i * x_i      (f32: one product, then one sum)
 * for a Normal term whose `affine` field is k + 1 (affines[k]).  slope is
 * CONST or PSCALAR; x is DATA, PVEC or a GATHER; the term's own loc operand is
 * CONST, PSCALAR, DATA, PVEC or a GATHER.  A non-injective gather may only
 * be the loc itself with a DATA x (alpha[group] + beta * x: the segmented
 * tape); x's parameter range must not overlap another accumulating operand
 * of the term (MC_ERR_UNSUPPORTED otherwise).  Examples: a + b * x (linear
 * regression), mu + tau * z (non-centred hierarchy), alpha[g] + beta * x
 * (varying intercepts).  Affine programs run on the chain-per-workgroup
 * kernels (k_hmc, k_nuts, k_mh).                                            */
typedef struct mc_affine {
    mc_operand slope, x;
} mc_affine;

/* Expression terms (MC_DIST_EXPR).  The reference differentiates ANY MLX
 * expression of the parameters (hmc.py:53-67 mx.grad over the user's
 * log_prob, nuts.py:76-87); the fused terms above cover the distribution
 * shapes, and an expression term covers everything else that is elementwise:
 *     weight * sum_i root_i
 * where the term's nodes form a DAG evaluated per broadcast element i in f32
 * (MLX's elementwise ops, each rounded once) and differentiated in reverse
 * mode with the VJPs mx.grad uses.  Node k's arguments are nodes of the same
 * term with smaller indices (a, b, c; -1 = unused); the last node is the
 * root.  Leaves are mc_operands: CONST, PSCALAR, DATA, PVEC or GATHER
 * (transform MC_XF_NONE — mx.exp / mx.log are nodes here).  Vector leaves
 * have the term's length n.  Every non-injective GATHER leaf of a term must
 * use the same index values (e.g. alpha[g] + beta[g] * x): the term is then
 * evaluated per group run (segmented, deterministic); anything else is
 * strided.  A term holds at most MC_EXPR_MAX_NODES nodes.                 */
#define MC_EXPR_MAX_NODES 32
typedef enum {
    MC_EX_LEAF    = 0,   /* the node's operand                               */
    MC_EX_ADD     = 1,   /* a + b                                            */
    MC_EX_SUB     = 2,   /* a - b                                            */
    MC_EX_MUL     = 3,   /* a * b                                            */
    MC_EX_DIV     = 4,   /* a / b                                            */
    MC_EX_NEG     = 5,   /* -a                                               */
    MC_EX_EXP     = 6,   /* exp a                                            */
    MC_EX_LOG     = 7,   /* log a                                            */
    MC_EX_SQRT    = 8,   /* sqrt a                                           */
    MC_EX_SQUARE  = 9,   /* a * a                                            */
    MC_EX_POW     = 10,  /* a ** b                                           */
    MC_EX_ABS     = 11,  /* |a|                                              */
    MC_EX_LOG1P   = 12,  /* log(1 + a)                                       */
    MC_EX_TANH    = 13,  /* tanh a                                           */
    MC_EX_SIGMOID = 14,  /* 1 / (1 + exp(-a))                                */
    MC_EX_NORMAL_LP      = 15,  /* Normal(b, c).log_prob(a)  normal.py:49-56 */
    MC_EX_HALFNORMAL_LP  = 16,  /* HalfNormal(c).log_prob(a) halfnormal.py:43-63 */
    MC_EX_EXPONENTIAL_LP = 17,  /* Exponential(c).log_prob(a) exponential.py:48-71 */
    MC_EX_WHERE   = 18,  /* a != 0 ? b : c, a a CONST / DATA leaf or a       */
                         /* comparison node (mx.where over a data mask or a  */
                         /* traced condition; no cotangent through a)        */
    MC_EX_GAMMA_LP = 19, /* Gamma(b, c).log_prob(a)  gamma.py:48-88: gammaln */
                         /* (b) at the current value, no cotangent through it */
    MC_EX_BETA_LP  = 20, /* Beta(b, c).log_prob(a)   beta.py:45-91: log B(b, */
                         /* c) at the current values, no cotangent through it */
    MC_EX_GT       = 21, /* a > b  as 1 / 0 (mx.greater: a mask, no cotangent) */
    MC_EX_GE       = 22, /* a >= b                                           */
    MC_EX_LT       = 23, /* a < b                                            */
    MC_EX_LE       = 24  /* a <= b                                           */
} mc_expr_op;

typedef struct mc_expr_node {
    int32_t    op;         /* mc_expr_op                                    */
    int32_t    a, b, c;    /* argument nodes (index within the term), or -1 */
    mc_operand leaf;       /* MC_EX_LEAF                                    */
} mc_expr_node;

/* The nodes of one expression term: nodes[first .. first + count). */
typedef struct mc_expr {
    int32_t first, count;
} mc_expr;

typedef struct mc_program mc_program;

/* Build a program.  data / index are HOST arrays; the library copies them to
 * the device (and, for terms that gather through an unsorted index, stores a
 * permuted copy so that every term is processed in index order — this is what
 * makes the gather gradient a deterministic segmented sum).  Validates every
 * operand range.  lp_const is added to the total log density.              */
int mc_program_create(const mc_term* terms, int32_t n_terms, int32_t n_params,
                      float lp_const,
                      const float* data, int64_t n_data,
                      const int32_t* index, int64_t n_index,
                      mc_program** out);
/* mc_program_create ignores mc_term.affine (formerly reserved0); only
 * mc_program_create_affine reads it, so zero-initialise it there.          */
/* mc_program_create with affine loc operands (affines[0 .. n_affines)).    */
int mc_program_create_affine(const mc_term* terms, int32_t n_terms,
                             const mc_affine* affines, int32_t n_affines,
                             int32_t n_params, float lp_const,
                             const float* data, int64_t n_data,
                             const int32_t* index, int64_t n_index,
                             mc_program** out);
/* mc_program_create_affine with expression terms: a term whose dist is
 * MC_DIST_EXPR names exprs[k] through its `affine` field (k + 1) and leaves
 * value / loc / scale MC_OP_NONE.  Expression programs run on the
 * chain-per-workgroup kernels (k_hmc, k_nuts, k_mh, mc_logp_grad); the
 * sliced planners decline them.                                           */
int mc_program_create_expr(const mc_term* terms, int32_t n_terms,
                           const mc_affine* affines, int32_t n_affines,
                           const mc_expr* exprs, int32_t n_exprs,
                           const mc_expr_node* nodes, int32_t n_nodes,
                           int32_t n_params, float lp_const,
                           const float* data, int64_t n_data,
                           const int32_t* index, int64_t n_index,
                           mc_program** out);
int mc_program_destroy(mc_program* prog);
int32_t mc_program_num_params(const mc_program* prog);
/* The launch geometry the engine picked: waves per chain (1, 4 or 16).     */
int32_t mc_program_waves_per_chain(const mc_program* prog);

/* Sliced layout (HMC only; hmc.py:7-206 with a different work split).  A
 * program whose terms each have at most one per-element parameter operand
 * can be split into S data slices: parameters touched by one slice only
 * become private to it, broadcast parameters are replicated, and one
 * workgroup evaluates one slice for a block of 8 or 16 chains; the slices of
 * a block exchange their log p / broadcast-cotangent / kinetic partials once
 * per leapfrog step.  Results equal the chain-per-workgroup kernel's up to
 * fp32 summation order and do not depend on how chains are split over
 * launches or GPUs.  num_slices: 0 = automatic (the default chosen by
 * mc_program_create: 16 for >= 65536 elements, 8 for >= 16384, 4 for >= 2048
 * when the lane-resident kernel takes the layout, else unsliced — and then
 * planned as ONE slice of the lane-resident kernel when it qualifies),
 * 1 = off (the chain-per-workgroup kernel k_hmc), 2..64 = that many
 * (MC_ERR_UNSUPPORTED if the program does not qualify).  NUTS, MH,
 * mc_logp_grad and mc_state_init always use the chain-per-workgroup kernels. */
int mc_program_set_slices(mc_program* prog, int32_t num_slices);
int32_t mc_program_num_slices(const mc_program* prog);
/* Which kernel runs a sliced HMC program.  kernel: 0 = automatic (the
 * lane-resident kernel when the layout qualifies: <= 16 slices, <= 4
 * broadcast parameters, <= 256 private parameters per slice, every
 * per-element parameter operand private; else the term interpreter),
 * 1 = term interpreter, 2 = lane-resident (MC_ERR_UNSUPPORTED if the layout
 * does not qualify; mc_last_error says why).  mc_program_slice_kernel returns
 * the kernel a launch with L > 0 will use: 0 unsliced, 1 interpreter, 2
 * lane-resident.  Both compute the same sampler; they differ in fp32
 * summation order only.  On an unsliced program, 2 plans it as one slice of
 * the lane-resident kernel (no exchange; an error if it does not qualify), 0
 * does so when it qualifies and 1 keeps k_hmc.  mc_program_set_slices resets
 * the choice's layout.                                                      */
int mc_program_set_slice_kernel(mc_program* prog, int32_t kernel);
int32_t mc_program_slice_kernel(const mc_program* prog);
/* 1 when a lane-resident launch of this program runs the fast-form kernel
 * k_hmc_lf (every slice term a swept N(theta[g], scale) term over data or a
 * direct theta ~ N(loc, scale) term, every scalar term the own prior of a
 * broadcast parameter; MC_LANES_FAST=0 in the environment turns it off),
 * 0 when it runs k_hmc_lr or no lane-resident kernel, -1 on a null program. */
int32_t mc_program_lanes_fast(const mc_program* prog);
/* Why the program's HMC launches do not run the lane-resident kernel (e.g.
 * "lane-resident kernel: more than 4 broadcast parameters"), or "" when they
 * do or no plan was attempted; valid until the next set_slices /
 * set_slice_kernel / destroy.  The chain-per-workgroup and interpreter
 * kernels are 2-4x slower on programs the automatic plan would slice: the
 * Python driver turns a non-empty note on such a program into a warning. */
const char* mc_program_kernel_note(const mc_program* prog);
/* 1 when mc_nuts_run with this max_tree_depth runs the lane-resident NUTS
 * kernel k_nuts_lr (a program planned as one lane-resident slice; its arena
 * fits LDS; MC_NUTS_LANES=0 in the environment turns it off), 2 when it runs
 * its register-only variant (no broadcast parameter, no scalar term, one
 * Normal term with at most one element per parameter and a data or constant
 * scale: the gradient from per-parameter registers), 0 when it runs k_nuts,
 * 3 when it runs the sliced NUTS kernel k_nuts_sl (a program sliced onto the
 * fast-form lane layout of k_hmc_lf: one chain per wave per slice, one record
 * exchange per leaf; max_tree_depth <= 12 and the LDS arenas fit), -1 on a
 * null program.  All take the reference's decisions; they differ in fp32
 * summation order only.                                                     */
int32_t mc_program_nuts_lanes(const mc_program* prog, int32_t max_tree_depth);

/* Batched tape evaluation: for every point p, logp[p] = log density at
 * q[p, :] and grad[p, :] = its gradient (replaces hmc.py:53-67 mx.grad).   */
int mc_logp_grad(const mc_program* prog, int64_t n_points,
                 const float* q_dev, float* logp_dev, float* grad_dev,
                 void* hip_stream);

/* Elementwise Distribution.log_prob (normal.py:33-56, halfnormal.py:34-63,
 * exponential.py:48-71, gamma.py:61-88, beta.py:59-91):
 * out[i] = log_prob(value[i]; loc|alpha[i|0], scale|rate|beta[i|0]).  The
 * middle operand may be NULL for HalfNormal and Exponential.  *_bcast = 1
 * means the operand is a single element.                                    */
int mc_dist_log_prob(int32_t dist, int64_t n,
                     const float* value_dev, int32_t value_bcast,
                     const float* loc_dev, int32_t loc_bcast,
                     const float* scale_dev, int32_t scale_bcast,
                     float* out_dev, void* hip_stream);

/* ---- per-chain state ---------------------------------------------------- */
/* State blob layout (device memory, mc_state_bytes(prog, C) bytes):
 *   [mc_chain_scalars x C][pad to 256 B][q: C x D f32][pad][g: C x D f32]
 * mc_state_offsets() returns the byte offsets of q and g.                  */
typedef struct mc_chain_scalars {
    double  step_size;      /* epsilon (Python float in the reference)      */
    double  step_size_bar;  /* NUTS dual averaging epsilon_bar (nuts.py:64) */
    double  h_bar;          /* NUTS dual averaging H_bar (nuts.py:65)       */
    double  alpha_sum;      /* NUTS: sum of per-iteration accept stats      */
    float   mu;             /* NUTS: f32 log(10*eps0) (nuts.py:63)          */
    float   logp;           /* log density at the current position          */
    int32_t n_accept;       /* accepted (HMC) / alpha>0.5 (NUTS) this phase */
    int32_t n_total;        /* iterations in this phase                     */
    int32_t warmup_accept;  /* counters frozen at the warmup->sampling edge */
    int32_t warmup_total;
    int64_t depth_sum;      /* NUTS: sum of tree depths this phase          */
    int64_t warmup_depth_sum;
    int64_t n_grad;         /* gradient evaluations so far                  */
    int32_t n_divergent;    /* NUTS: leaves that failed the DELTA_MAX test  */
    int32_t reserved;
} mc_chain_scalars;

int64_t mc_state_bytes(const mc_program* prog, int64_t num_chains);
int mc_state_offsets(const mc_program* prog, int64_t num_chains,
                     int64_t* q_offset, int64_t* g_offset);
/* Set q = q0, evaluate logp/grad there, step_size = eps0, counters = 0,
 * NUTS dual-averaging state = (mu = f32 log(10 eps0), eps_bar = 1, H_bar = 0)
 * (nuts.py:62-68, hmc.py:157).                                              */
int mc_state_init(const mc_program* prog, int64_t num_chains,
                  const float* q0_dev, double step_size,
                  void* state_dev, void* hip_stream);

/* ---- sampling runs ------------------------------------------------------ */
/* Iterations are numbered globally: [0, num_warmup) is warmup, then
 * [num_warmup, num_warmup + num_samples) is sampling.  A launch runs
 * iterations [iter_begin, iter_begin + iter_count) for every chain, so a run
 * may be split over several launches (progress printing, bench steps).
 * Draws are a pure function of (seed, chain_offset + chain, iteration, ...),
 * so results do not depend on how chains are split over launches or GPUs. */
typedef struct mc_run_config {
    int64_t  num_chains;       /* chains in this launch                      */
    int64_t  chain_offset;     /* global index of chain 0 (RNG stream id)    */
    int64_t  num_warmup;
    int64_t  num_samples;
    int64_t  iter_begin;
    int64_t  iter_count;
    int64_t  sample_begin;     /* samples buffer holds sample indices        */
    int64_t  sample_capacity;  /*   [sample_begin, sample_begin + capacity)  */
    uint64_t seed;
    double   step_size;        /* initial epsilon (NUTS mu uses it)          */
    double   target_accept;
    int32_t  num_leapfrog_steps; /* HMC L                                    */
    int32_t  max_tree_depth;     /* NUTS                                     */
    int32_t  adapt_step_size;
    int32_t  slice_mode;         /* NUTS: 0 = reference f32 exp/log (Q7),    */
                                 /*       1 = exact double log u             */
} mc_run_config;

/* Optional per-(chain, iteration) trace; any pointer may be NULL.
 * Arrays are [num_chains, capacity] for iterations [iter_begin, +capacity). */
typedef struct mc_trace {
    int64_t  iter_begin;
    int64_t  capacity;
    uint8_t* accepted;      /* HMC accept bit; NUTS alpha > 0.5             */
    float*   accept_stat;   /* HMC log-accept ratio; NUTS alpha (nuts.py:287) */
    double*  step_size;     /* epsilon used in the iteration                */
    float*   energy;        /* HMC H_init; NUTS H0                          */
    int32_t* tree_depth;    /* NUTS j; HMC L                                */
    int32_t* n_leapfrog;    /* leapfrog steps (= new gradient evaluations)  */
} mc_trace;

/* HMC (hmc.py:7-206).  samples_dev: [num_chains, sample_capacity, D] f32 or
 * NULL.  workspace: mc_hmc_workspace_bytes() bytes of device memory (may be
 * 0 bytes when the per-chain arena fits in LDS).                            */
int64_t mc_hmc_workspace_bytes(const mc_program* prog, int64_t num_chains);
/* The lane-resident kernel continues its exchange tags across launches on a
 * workspace and clears the workspace only the first time it sees its address
 * (and after another kernel used it or a timeout was reported).  A caller
 * that frees or repurposes a workspace between sliced HMC launches calls
 * mc_workspace_release(ws) first.                                           */
int mc_workspace_release(const void* workspace_dev);

/* Test hook for the exchange kernels' timeout path (no reference counterpart):
 * while on != 0, the last workgroup of every sliced HMC launch exits without
 * publishing, so the other slices of its chain block time out;
 * mc_workspace_status then reports MC_ERR_TIMEOUT and the next launch on the
 * workspace starts clean.  The state of a timed-out chain block is undefined
 * in general and the caller re-initialises those chains: the HMC and MH
 * kernels write a chain's state only at launch exit (a stranded block keeps
 * the state the launch found), but sliced NUTS writes an accepted draw's
 * private parameters when its tree level completes, and its shared
 * parameters, log density and scalars at exit (csrc/nuts_sliced.h).  The
 * hook faults before the first leaf, where every kernel keeps the state.  */
int mc_debug_exchange_fault(int on);
/* Test hook: 0 runs the fast-form kernel k_hmc_lf with the term form read at
 * run time (FORM = -1) instead of its compile-time instantiations; 1 restores
 * the default.  Results agree up to fp32 summation order.                  */
int mc_debug_lanes_forms(int on);
/* Test hook: 0 runs every lane-resident HMC launch on the general kernel
 * k_hmc_lr instead of the fast-form k_hmc_lf (as MC_LANES_FAST=0 in the
 * environment); 1 restores the default.  Results agree up to fp32
 * summation order.                                                        */
int mc_debug_lanes_fast(int on);
/* Test hook for k_nuts_lr's variants: -1 (default) picks the fastest variant
 * the program qualifies for; 0 forces the generic lane evaluator (SPEC 0);
 * 1 forces the specialised variant (SPEC 1) where the program qualifies,
 * skipping the register-only one.  Trees agree up to fp32 summation order. */
int mc_debug_nuts_variant(int variant);
/* Test hook for the sliced NUTS kernel k_nuts_sl (csrc/nuts_sliced.h): 0
 * runs sliced fast-form programs on k_nuts (the tape) instead, 1 on k_nuts_sl,
 * -1 restores the default (MC_NUTS_SLICED from the environment, else on).
 * Trees agree up to fp32 summation order.                                  */
int mc_debug_nuts_sliced(int on);
/* Diagnostic of the same-XCD exchange (csrc/sliced.h xcd_announce /
 * xcd_agree): the exchange groups (chain blocks, counted by their slice 0)
 * launched on `ws` since it was last cleared whose slices all sat on one XCD
 * (their records then stay in that XCD's L2), and those whose did not.      */
int mc_debug_workspace_xcd(const void* ws, int32_t* local, int32_t* remote);
/* The same-XCD exchange (L2-resident records, csrc/host.h xcd_round_robin):
 * 0 off, 1 on where the device's workgroup placement allows it, -1 the
 * default (MC_XCD_LOCAL from the environment, else on).  Results are the same
 * bits either way.                                                          */
int mc_debug_xcd_local(int on);
/* The sliced Metropolis-Hastings kernel k_mh_sl (csrc/mh_sliced.h):
 * mc_program_mh_sliced is 1 when mc_mh_run runs it (a program sliced onto
 * the fast-form lane layout: one wave per chain and slice, one log-p record
 * exchange per iteration), 0 when it runs k_mh on the tape, -1 on a null
 * program; mc_debug_mh_sliced: 0 forces k_mh, 1 allows k_mh_sl, -1 the
 * default (MC_MH_SLICED from the environment, else on).                    */
int32_t mc_program_mh_sliced(const mc_program* prog);
int mc_debug_mh_sliced(int on);
/* Expression terms (MC_DIST_EXPR) compiled per program (csrc/jit.hip):
 * hiprtc compiles the tape kernels' expression instantiations with each
 * term's node DAG as straight-line code (the interpreter's operations in its
 * order: bit-identical results), at the first launch that needs them; code
 * objects are cached per structure in the process and on disk ($MC_JIT_CACHE,
 * else ~/.cache/mcmc355).  mc_debug_expr_jit: 0 keeps the interpreter, 1 the
 * JIT, -1 the default (MC_EXPR_JIT from the environment, else on).
 * mc_program_expr_jit: 1 when the program's expression terms run compiled,
 * 0 when it has none or the JIT is off, -2 when their compilation failed (the
 * interpreter runs; mc_program_kernel_note says why), -1 on a null program. */
int mc_debug_expr_jit(int on);
int32_t mc_program_expr_jit(const mc_program* prog);
/* Test hooks without a device: mc_debug_program_host_only(1) makes the next
 * programs built on this thread host tables only (never launch them);
 * mc_debug_expr_jit_source copies the generated source of a program's
 * expression terms (returns its length); mc_debug_expr_jit_compile compiles
 * it into `kernel` (e.g. "mc::k_hmc<8, true, true>"), MC_OK or the
 * compiler's log as the error.                                              */
int mc_debug_program_host_only(int on);
int64_t mc_debug_expr_jit_source(const mc_program* prog, char* buf, int64_t cap);
int mc_debug_expr_jit_compile(const mc_program* prog, const char* kernel);
/* Test hook without a device: plan a host-only program's S slices onto the
 * lane-resident layout (host tables only); with expression terms on it,
 * mc_debug_expr_jit_source / _compile take a "mc::k_hmc_lr<...>" kernel name
 * and give / compile the lane-resident source (jit.hip gen_lane_source).  */
int mc_debug_lane_plan_host(mc_program* prog, int32_t num_slices);
int64_t mc_debug_expr_jit_lane_source(const mc_program* prog, char* buf, int64_t cap);
/* Test hooks (host code, no device): the samplers' Box-Muller pair from two
 * Philox words per pair (words [n][2] -> out [n][2] f32) and their f32 log
 * of a uniform in (0, 1] (philox.h mc_box_muller / mc_logf_unit).         */
int mc_box_muller_host(const uint32_t* words, int64_t n, float* out);
int mc_logf_unit_host(const float* x, int64_t n, float* out);
/* After a sliced mc_hmc_run: MC_OK, or MC_ERR_TIMEOUT if an exchange timed
 * out (the launch then left its chains' state unchanged or partial).
 * Synchronises the stream.  Always MC_OK for an unsliced program.         */
int mc_workspace_status(const mc_program* prog, const void* workspace_dev,
                        int64_t workspace_bytes, void* hip_stream);
int mc_hmc_run(const mc_program* prog, const mc_run_config* cfg,
               void* state_dev, float* samples_dev, const mc_trace* trace,
               void* workspace_dev, int64_t workspace_bytes, void* hip_stream);

/* NUTS (nuts.py:16-358), iterative tree building, max_tree_depth <= 16.    */
int64_t mc_nuts_workspace_bytes(const mc_program* prog, int64_t num_chains,
                                int32_t max_tree_depth);
int mc_nuts_run(const mc_program* prog, const mc_run_config* cfg,
                void* state_dev, float* samples_dev, const mc_trace* trace,
                void* workspace_dev, int64_t workspace_bytes, void* hip_stream);

/* Random-walk Metropolis-Hastings (metropolis.py:6-101): per iteration
 * q' = q + f32(z * f32(proposal_scale)), z ~ N(0, I) (Philox, tag
 * MC_RNG_TAG_PROPOSAL), accept iff f32 log U < f32(lp(q') - lp(q)) (NaN
 * rejects), the current point is stored after every iteration.  The forward
 * tape only: one log density evaluation per iteration.  Every iteration of
 * the launch is a sampling iteration (set num_warmup = 0; MCMC.run's warmup
 * is a separate sampler run with its own seed, mcmc.py:145-178).  Uses
 * num_chains, chain_offset, iter_begin/iter_count, sample_begin/capacity and
 * seed of cfg; the state's logp (mc_state_init) is the current log density.
 * The gradient section of the state is not updated.  Trace: accepted,
 * accept_stat = log ratio, step_size = proposal scale, energy = log p.      */
int64_t mc_mh_workspace_bytes(const mc_program* prog, int64_t num_chains);
int mc_mh_run(const mc_program* prog, const mc_run_config* cfg, double proposal_scale,
              void* state_dev, float* samples_dev, const mc_trace* trace,
              void* workspace_dev, int64_t workspace_bytes, void* hip_stream);

/* ---- RNG (replaces mx.random for the sampler draws) --------------------- */
/* Philox4x32-10 (Salmon et al., SC'11).  key = (seed lo, seed hi); counter =
 * (chain, iteration, tag << 24 | sub, index).  mode 0: raw u32 words
 * (out is uint32[n*4]); 1: f32 uniforms in (0,1) ((w >> 9) + 0.5) 2^-23;
 * 2: f32 standard normals, double-precision Box-Muller on word pairs.
 * Element e uses counter (chain, iteration, tag<<24 | sub, index0 + e).     */
#define MC_RNG_TAG_MOMENTUM 1
#define MC_RNG_TAG_ACCEPT   2
#define MC_RNG_TAG_SLICE    3
#define MC_RNG_TAG_DEPTH    4
#define MC_RNG_TAG_MERGE    5
#define MC_RNG_TAG_PROPOSAL 6   /* Metropolis-Hastings random-walk noise      */
#define MC_RNG_TAG_USER     16
int mc_rng_fill(uint64_t seed, uint32_t chain, uint32_t iteration,
                uint32_t tag, uint32_t sub, uint32_t index0, int64_t n,
                int32_t mode, void* out_dev, void* hip_stream);

/* ---- diagnostics over a sample buffer [C, S, D] (device, f32) ---------- */
/* A series is samples[c, :, d].  mc_series_stats writes stats[f * C*D + c*D + d]
 * (f64, device) for each field f:                                            */
#define MC_ST_ESS     0   /* compute_ess (examples/06_nuts_comparison.py:22-41):
                             n / (1 + 2 sum rho_k), lags 1 .. min(S/2, max_lag)-1,
                             stopping at (and including) the first rho < 0.05;
                             S when the variance is 0.  max_lag = 100 there.  */
#define MC_ST_MEAN    1   /* series mean                                      */
#define MC_ST_M2      2   /* sum of squared deviations from the mean          */
#define MC_ST_HMEAN0  3   /* mean of draws [0, S/2)                           */
#define MC_ST_HMEAN1  4   /* mean of draws [S - S/2, S)                       */
#define MC_ST_HM2_0   5   /* sum of squared deviations, first half            */
#define MC_ST_HM2_1   6   /* sum of squared deviations, second half           */
#define MC_ST_COUNT   7
int mc_series_stats(int64_t C, int64_t S, int64_t D, const float* samples_dev,
                    int32_t max_lag, double* stats_dev, void* hip_stream);
/* Chain-order reduction to out_dev[2, D] (f64).  center_dev == NULL:
 *   out[0][d] = sum of the 2C half-chain means, out[1][d] = sum_c ESS.
 * center_dev = that out[0] summed over every rank (m_total = all half chains):
 *   out[0][d] = sum (half mean - center[d]/m_total)^2,
 *   out[1][d] = sum of half-chain variances (ddof 1).
 * Multi-GPU: all-reduce (sum) out between the two calls and after the second. */
int mc_stats_reduce(int64_t C, int64_t S, int64_t D, const double* stats_dev,
                    const double* center_dev, int64_t m_total, double* out_dev,
                    void* hip_stream);
/* Split R-hat (Gelman et al., BDA3 eq. 11.4) over m_total half chains of
 * S/2 draws from the second reduction: rhat_dev[D] (f64).  S >= 4.          */
int mc_rhat(int64_t D, int64_t m_total, int64_t S, const double* spread_dev,
            double* rhat_dev, void* hip_stream);
/* Pooled mean and std (ddof 0) of every value of elements [off, off+len)
 * over all chains and draws (mcmc.py:205-206): out_dev[2] f64.             */
int mc_pool_moments(int64_t C, int64_t S, int64_t D, const double* stats_dev,
                    int64_t off, int64_t len, double* out_dev, void* hip_stream);
/* Exact order statistics (0-based ranks k[0..nk), host array, nk <= 8) of the
 * pooled values of elements [off, off+len): out_dev[nk] f32; NaN if any
 * pooled value is NaN (np.percentile / np.median, mcmc.py:207-209).          */
int64_t mc_select_workspace_bytes(int32_t nk);
int mc_select(int64_t C, int64_t S, int64_t D, const float* samples_dev,
              int64_t off, int64_t len, int32_t nk, const int64_t* k,
              float* out_dev, void* workspace_dev, int64_t workspace_bytes,
              void* hip_stream);

const char* mc_last_error(void);
int32_t mc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MCMC355_H */
