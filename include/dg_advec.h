/*
 * dg_advec.h — C ABI of the MI355X-native forward + adjoint DG advection time-stepper.
 *
 * The reference (wglao/Adjoint-ODE-Adaptivity) has no FFI: its hot path is a set of
 * MATLAB global-state functions (utils/AdvecRHS1D.m, utils/SlopeLimitN.m, utils/minmod.m),
 * an inlined LSERK4 loop (utils/One_code.mlx:106-140) and the DWR/refine pattern of
 * python/Main_finite_difference.py:54-94,336-341.  Each entry point below names the
 * reference interface it replaces.  A Python caller binds it with ctypes
 * (adjoint-ode-adaptivity_amd/_lib.py; stub in INTEGRATION.md).
 *
 * Conventions
 *  - Layout: element-major fp64, u[e*Np + i] with e = b*K + k (trajectory b, element k),
 *    byte-identical to MATLAB's Np x K column-major array for one trajectory.
 *  - All array arguments of compute calls are DEVICE pointers owned by the caller.  The
 *    library never frees caller memory and never allocates inside compute calls; scratch
 *    lives in the plan.  Host pointers appear only in dg_plan_create (copied).
 *  - Every function returns 0 (DG_OK) or a negative DG_ERR_* code; dg_last_error() gives
 *    the message of the last failure on the calling thread.  No exception crosses the ABI.
 *  - Compute calls are asynchronous on `stream` (a hipStream_t, NULL = default stream);
 *    the caller synchronises.  A plan may be shared by threads that use different streams
 *    for dg_advec_rhs / dg_slope_limit_n; dg_lserk4_fwd / dg_lserk4_adj / dg_argmax use
 *    plan scratch and must not run concurrently on one plan.
 */
#ifndef DG_ADVEC_H
#define DG_ADVEC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dg_plan dg_plan;

enum {
  DG_OK = 0,
  DG_ERR_ARG = -1,         /* invalid argument (null pointer, bad size, unsupported N) */
  DG_ERR_HIP = -2,         /* a HIP runtime call failed (message has hipGetErrorString) */
  DG_ERR_NOMEM = -3        /* device allocation failed in dg_plan_create */
};

/* Inflow boundary value at x = 0.
 *   DG_INFLOW_SIN_AT : uin = -sin(a*t)    utils/AdvecRHS1D.m:14
 *   DG_INFLOW_SIN_A2T: uin = -sin(a*a*t)  utils/One_code.mlx:129 (the executed golden run)
 *   DG_INFLOW_ZERO   : uin = 0            the homogeneous problem (a pulse leaving the domain:
 *                                         exact solution u0(x - a t); the effectivity study) */
enum { DG_INFLOW_SIN_AT = 0, DG_INFLOW_SIN_A2T = 1, DG_INFLOW_ZERO = 2 };

/* Time integrator of the forward step and of its discrete adjoint.
 *   DG_TIME_LSERK4: 5-stage low-storage RK4, coefficients utils/Globals1D.m:19-34
 *   DG_TIME_EULER : forward Euler u += dt*rhs (config 1 plumbing, Main_finite_difference.py:131-132 pattern) */
enum { DG_TIME_LSERK4 = 0, DG_TIME_EULER = 1 };

/* Last error message of the calling thread ("" if none). */
const char* dg_last_error(void);

/* Library version string. */
const char* dg_version(void);

/* Create an immutable plan (replaces the MATLAB globals set by utils/StartUp1D.m:5-39 and
 * utils/Globals1D.m:3-34, and the python/galerkin.py:199-237 startUp1D attribute set).
 *   N       polynomial order, 1..8 (Np = N+1 nodes per element)
 *   K       elements per trajectory;  batch  independent trajectories (ensemble ICs) sharing the mesh
 *   r, V, invV, Dr, LIFT   host arrays from the host setup (JacobiGL/Vandermonde1D/Dmatrix1D/Lift1D):
 *           r[Np], V/invV/Dr row-major [Np][Np], LIFT row-major [Np][2]
 *   VX      host array of K+1 vertex coordinates (utils/MeshGen1D.m:4-14, or a refined mesh)
 *   a       advection speed; inflow_variant DG_INFLOW_*; time_scheme DG_TIME_*
 * The metric rx = Fscale = 2/h_k is taken per element from VX (uniform meshes use one scalar). */
int dg_plan_create(int N, int64_t K, int64_t batch,
                   const double* r, const double* V, const double* invV,
                   const double* Dr, const double* LIFT, const double* VX,
                   double a, int inflow_variant, int time_scheme, dg_plan** out);

/* Destroy a plan (frees its device scratch).  NULL is a no-op. */
int dg_plan_destroy(dg_plan* plan);

/* Query plan sizes: out[0]=N, out[1]=Np, out[2]=K, out[3]=batch, out[4]=uniform mesh (0/1),
 * out[5]=time stages per step, out[6]=tile width, out[7]=time steps per launch. */
int dg_plan_query(const dg_plan* plan, int64_t out[8]);

/* Tuning knobs of the fused step kernels.  Tile width and tile order leave the arithmetic
 * bit-identical; steps per launch changes it at rounding level only.
 *   DG_TUNE_TILE_WIDTH        1 or 2: workgroups of 256*value lanes, one element per lane,
 *                             own tiles of 256*value elements (2: half the halo overhead)
 *   DG_TUNE_STEPS_PER_LAUNCH  time steps fused per launch: 1, 2, 4 or 8 (temporal blocking:
 *                             each launch reads its input state once and writes every
 *                             intermediate snapshot; halo = steps*stages elements per side;
 *                             8 needs tile width 2, else 4 is used; Np = 9 caps it at 2)
 *   DG_TUNE_XCD_ORDER         0/1: give each XCD a contiguous range of tiles (speed only)
 *   DG_TUNE_LANE_ELEMENTS     0: workgroup tiles, one element per lane; 2 or 4: forward steps
 *                             on one-wave tiles of 64*value elements, value consecutive
 *                             elements per lane, cross-lane faces by DPP (LSERK4, Np <= 8;
 *                             bit-identical to the workgroup tiles at equal steps per launch)
 *   DG_TUNE_REC_TILE_WIDTH    1 or 2: tile width of the jump-record sweeps, both directions
 *                             (dg_lserk4_fwd_rec / dg_lserk4_adj_rec): workgroups of 256*value
 *                             lanes (default 2; at Np = 9 1 for the adjoint, 2 for the forward)
 *   DG_TUNE_REC_FWD_TILE_WIDTH  the forward record sweep's own tile width (0: as the adjoint's)
 *   DG_TUNE_REC_STEPS_PER_LAUNCH  their steps per launch, both directions (default 10): 1, 2,
 *                             4, 5, 8, 10, 16
 *                             or 20 on pair tiles (16 and 20 need tile width 2, else 8 / 10
 *                             are used), a sweep chunked by halving (20 -> 10 -> 5 -> 2 -> 1);
 *                             1, 2, 4 or 8 on one element per lane (8 needs tile width 2,
 *                             else 4; Np = 9 caps those at 2)
 *   DG_TUNE_REC_FWD_STEPS_PER_LAUNCH  the forward record sweep's own steps per launch (same
 *                             values; default by size: 20 on 1024-element pair tiles up to
 *                             3*2^20 elements per plan, else as the adjoint; setting
 *                             DG_TUNE_REC_STEPS_PER_LAUNCH makes it "as the adjoint")
 *   DG_TUNE_REC_LANE_ELEMENTS 1 or 2: consecutive elements per lane of the jump-record sweeps'
 *                             workgroup tiles (default 2: tiles of 512*width elements,
 *                             lane-internal faces in registers; bit-identical to 1 at
 *                             equal steps per launch)
 *   DG_TUNE_REC_SWEEP         1 (default): dg_lserk4_sweep_rec runs forward and adjoint as one
 *                             dataflow launch where the record shape allows it; 0: as the
 *                             launch-per-block pair dg_lserk4_fwd_rec + dg_lserk4_adj_rec
 *   DG_TUNE_P_TILE_WIDTH      1 or 2: tile width of the p-enriched estimate (dg_lserk4_adj_p):
 *                             workgroups of 256*value lanes, one element per lane (default 2)
 *   DG_TUNE_P_STEPS_PER_LAUNCH its steps per launch: 1, 2, 4 (default) or 8 (8 needs tile
 *                             width 2, else 4); a sweep is chunked by halving
 *   DG_TUNE_SWEEP_WAVES       workgroup waves of the dataflow sweep (dg_lserk4_sweep_rec): 0 (the
 *                             default: as the record sweeps' tile width, 4 or 8 waves, except
 *                             12 on uniform meshes at 3 <= Np <= 5 with 1024-element record tiles,
 *                             >= 10-step forward and 10-step adjoint blocks, and 8 on uniform
 *                             meshes at Np = 9), 4, 8, 12 or 16 (16 at
 *                             Np <= 5); tiles of 128 * waves elements in both directions, also
 *                             where the launch chains' forward and adjoint widths differ (12
 *                             and 16 take 10- or 20-step forward and 10-step adjoint blocks).
 *                             Bit-identical results at any value
 *   DG_TUNE_SWEEP_LANE_ELEMENTS  consecutive elements per lane of the dataflow sweep's tiles:
 *                             2 (default), or 4 at Np <= 3 on 4- or 8-wave workgroups (tiles
 *                             of 256 * waves elements: half the barriers per element, half the
 *                             halo share).  Bit-identical results
 *   DG_TUNE_SWEEP_TAKE        0 only: dataflow work items come from one take counter (round 4's
 *                             1, item = workgroup id, relied on in-order dispatch per XCD and
 *                             was removed in round 5; 1 is an argument error)
 *   DG_TUNE_SWEEP_EXCHANGE    how the dataflow sweep's tiles exchange element faces: 0 (default)
 *                             through LDS with a workgroup barrier per Horner level; 1
 *                             overlapped waves: faces within a wave by DPP, one LDS exchange of
 *                             6 ghost elements per wave end and one barrier per time step
 *                             (tiles of waves * 116 + 12 elements on 8, 12 or 16 (Np <= 5)
 *                             waves; 20- or 10-step forward and 10-step adjoint blocks).
 *                             Bit-identical results
 *   DG_TUNE_SNAP_PAIRS        dg_lserk4_fwd with snapshots: 0 (default) the stage-loop kernels
 *                             (bit-identical to the record sweeps' stage loop), 1 the Horner-form
 *                             step on pair tiles (512 * tile width elements, steps per launch as
 *                             DG_TUNE_STEPS_PER_LAUNCH; equal to the stage loop to rounding)
 *   DG_TUNE_P_FLOW            dg_lserk4_adj_p: 1 (default) runs the estimate as ONE dataflow launch (the
 *                             blocks' tiles are work items; the jump sweep's hand-offs and
 *                             watchdog) when nsteps splits into 2 .. 40/steps-per-launch blocks
 *                             of the plan's steps per launch; 0 one launch per block.
 *                             Bit-identical results
 *   DG_TUNE_P_SWEEP           dg_lserk4_sweep_p: 1 (default) runs the snapshot forward and the
 *                             estimate as ONE dataflow launch where dg_plan_query_p_sweep
 *                             allows; 0 the chains, whose forward runs at 4 steps per launch
 *                             like the launch's blocks.  Bit-identical results (a separate
 *                             dg_lserk4_fwd at another steps per launch rounds differently)
 *   DG_TUNE_NL_EXCHANGE       the config-3 kernels (nonlinear flux and/or per-stage limiter,
 *                             dg_lserk4_fwd(_ex) / dg_lserk4_adj(_ex)): 0 workgroup tiles
 *                             exchanging faces and cell averages through LDS with a barrier
 *                             each; 1 overlapped waves: every wave owns 44 of a 64-element
 *                             window, every exchange a DPP wave shift, no barrier inside a step
 *                             (one step per forward launch; the limited adjoint needs the
 *                             decision record, else it runs the workgroup tiles).
 *                             Bit-identical results
 *   DG_TUNE_SWEEP_SPIN_LIMIT  diagnostics/tests: polls a dataflow work item makes before it
 *                             gives up waiting for a producer (0: the default, ~2^20; 1 makes
 *                             the watchdog fire on any multi-block sweep)
 * Environment overrides at plan creation: DG_TILE_WIDTH, DG_STEPS_PER_LAUNCH, DG_LANE_ELEMENTS,
 * DG_REC_TILE_WIDTH, DG_REC_FWD_TILE_WIDTH, DG_REC_STEPS_PER_LAUNCH, DG_REC_FWD_STEPS_PER_LAUNCH, DG_REC_LANE_ELEMENTS,
 * DG_P_TILE_WIDTH, DG_P_STEPS_PER_LAUNCH, DG_SWEEP_WAVES, DG_SWEEP_LANE_ELEMENTS, DG_SWEEP_EXCHANGE, DG_SNAP_PAIRS, DG_P_FLOW, DG_P_SWEEP, DG_NL_EXCHANGE. */
enum { DG_TUNE_TILE_WIDTH = 1, DG_TUNE_STEPS_PER_LAUNCH = 2, DG_TUNE_XCD_ORDER = 3,
       DG_TUNE_LANE_ELEMENTS = 4, DG_TUNE_REC_TILE_WIDTH = 5, DG_TUNE_REC_STEPS_PER_LAUNCH = 6,
       DG_TUNE_REC_LANE_ELEMENTS = 7, DG_TUNE_REC_FWD_STEPS_PER_LAUNCH = 8,
       DG_TUNE_P_TILE_WIDTH = 9, DG_TUNE_P_STEPS_PER_LAUNCH = 10,
       DG_TUNE_REC_FWD_TILE_WIDTH = 11, DG_TUNE_REC_SWEEP = 12,
       DG_TUNE_SWEEP_SPIN_LIMIT = 13, DG_TUNE_SWEEP_WAVES = 14,
       DG_TUNE_SWEEP_LANE_ELEMENTS = 15, DG_TUNE_SWEEP_TAKE = 16, DG_TUNE_SWEEP_EXCHANGE = 17,
       DG_TUNE_SNAP_PAIRS = 18, DG_TUNE_P_FLOW = 19, DG_TUNE_P_SWEEP = 20,
       DG_TUNE_NL_EXCHANGE = 21 };
int dg_plan_tune(dg_plan* plan, int key, int64_t value);

/* The jump-record sweeps' effective shape: out[0] = tile width, out[1] = steps per launch
 * (adjoint), out[2] = elements per lane, out[3] = the forward's steps per launch. */
int dg_plan_query_rec(const dg_plan* plan, int64_t out[4]);

/* The forward record sweep's shape: out[0] = tile width, out[1] = steps per launch. */
int dg_plan_query_rec_fwd(const dg_plan* plan, int64_t out[2]);

/* The p-enriched estimate's effective shape: out[0] = tile width, out[1] = steps per launch. */
int dg_plan_query_p(const dg_plan* plan, int64_t out[2]);

/* The config-3 kernels' shape (nonlinear flux and/or limiter): out[0] = the exchange
 * (DG_TUNE_NL_EXCHANGE: 0 workgroup tiles, 1 overlapped waves), out[1] = forward steps per
 * launch with snapshots, out[2] = without. */
int dg_plan_query_nl(const dg_plan* plan, int64_t out[3]);

/* Physics of the plan's steppers.  Default: DG_FLUX_LINEAR + DG_LIMIT_NONE (AdvecRHS1D).
 *   DG_FLUX_LINEAR      f(u) = a*u                               utils/AdvecRHS1D.m:9-19
 *   DG_FLUX_BURGERS     f(u) = a*u^2/2 at the nodes with AdvecRHS1D's central-flux structure
 *                       on f and inflow f(uin) (build-defined, BASELINE config 3, SURVEY 8d;
 *                       CPU statement oracle/burgers.py)
 *   DG_LIMIT_EACH_STAGE u = SlopeLimitN(u) (utils/SlopeLimitN.m:1-33) after every stage update
 *   DG_LIMIT_PI1_EACH_STAGE  u = SlopeLimit1(u) (utils/SlopeLimit1.m:1-23, every cell limited)
 *                       after every stage update
 * Both need DG_TIME_LSERK4.  With either, dg_advec_rhs evaluates the flux's RHS (no limiter),
 * dg_lserk4_fwd runs limited steps (1 or 2 per launch), and dg_lserk4_adj is the exact
 * transpose of each step's tangent at the stored forward states, with the limiter's discrete
 * decisions (troubled cells, active minmod argument) frozen; it recomputes step n's stages from
 * snapshots[n] (one launch per step) and takes the indicator residual of the flux f. */
enum { DG_FLUX_LINEAR = 0, DG_FLUX_BURGERS = 1 };
enum { DG_LIMIT_NONE = 0, DG_LIMIT_EACH_STAGE = 1, DG_LIMIT_PI1_EACH_STAGE = 2 };
int dg_plan_set_physics(dg_plan* plan, int flux, int limiter);

/* Grow the plan's device mesh and scratch buffers to hold K_capacity elements per trajectory,
 * so that dg_plan_refine can add elements without reallocating.  Synchronous (waits for the
 * device); never shrinks; a no-op when the capacity suffices.  The dataflow sweep's scratch is
 * sized for the reserved capacity, so refines within it reuse it; a growing reserve frees the
 * plan's old scratch (also scratch regions earlier sweeps outgrew), so HIP graphs captured
 * before it must be re-captured. */
int dg_plan_reserve(dg_plan* plan, int64_t K_capacity);

/* Refine on the device: split element idx[0] (device int64 in [0, K), e.g. dg_argmax's
 * output) at its midpoint, i.e. insert 0.5*(VX[idx] + VX[idx+1]) after vertex idx — the split
 * of python/Main_finite_difference.py:336-341 (ref_idx = argmax + 1) and matlab/MAIN.m:137-141 —
 * with the new elements' metric 2/h as dg_plan_create computes it.  K grows by one and the
 * mesh is non-uniform from then on; fields sized for the old K must be re-initialised by the
 * caller (e.g. dg_init_sine).  h_split (nullable, device double) receives the width of the
 * split element.  Needs K+1 <= capacity (dg_plan_reserve).  Asynchronous on stream; the plan
 * is modified, so it must not be used concurrently. */
int dg_plan_refine(dg_plan* plan, const int64_t* idx, double* h_split, void* stream);

/* Copy the plan's current K+1 vertex coordinates to the host array VX (synchronous). */
int dg_plan_get_mesh(const dg_plan* plan, double* VX);

/* rhs = AdvecRHS1D(u, t, a)   — utils/AdvecRHS1D.m:1-20 (inline copy One_code.mlx:124-134).
 * Central flux (alpha = 1), inflow at each trajectory's x = 0, du = 0 at the outflow face. */
int dg_advec_rhs(const dg_plan* plan, const double* u, double* rhs, double t, void* stream);

/* Forward sweep: nsteps fused steps of the plan's integrator starting at time t0
 * (the "dg_march" role; LSERK4 loop One_code.mlx:106-140, time = time + dt as there).
 * u (in/out): the state.  snapshots (nullable): (nsteps+1) consecutive states,
 * snapshots[n] = u^n.  u may alias snapshots[0]: then u^0 is neither copied nor
 * overwritten (u keeps u^0) and the final state is snapshots[nsteps]. */
int dg_lserk4_fwd(dg_plan* plan, double* u, double t0, double dt, int nsteps,
                  double* snapshots, void* stream);

/* dg_lserk4_fwd that also records the per-stage limiter's decisions (plans with a per-stage
 * limiter only; ignored otherwise): decisions (nullable, device, nsteps*batch*K uint16) gets,
 * for step n and element e, decisions[n*batch*K + e] = sum over stages s of
 * code_s << (3 s), code_s = 0 (not troubled, SlopeLimitN.m:23) or 4 | (active minmod
 * argument 0..3, minmod.m:9-11).  dg_lserk4_adj_ex reads the record back. */
int dg_lserk4_fwd_ex(dg_plan* plan, double* u, double t0, double dt, int nsteps,
                     double* snapshots, uint16_t* decisions, void* stream);

/* Adjoint sweep + dual-weighted residual (the "adj_march" / "adjoint_sens" / "err_contribution"
 * role; discrete-adjoint pattern python/Main_finite_difference.py:54-76, indicator pattern :79-94).
 * Exact discrete transpose of the forward step, run for n = nsteps-1 .. 0:
 *   w^{n+1} += src_coef * u^{n+1}   (functional source, left-endpoint rule: none at n+1 = nsteps)
 *   eta[e]  += dt * sum_i w^{n+1}[e,i] * R(u^{n+1}, t_{n+1})[e,i]
 *              R = LIFT*(Fscale.*du): the interelement-jump (strong-form) residual of AdvecRHS1D
 *   w^n      = S^T w^{n+1}
 * and finally w^0 += src_coef * u^0.
 *   w (in/out): terminal dJ/du^N on entry, dJ/du^0 on exit.  w may alias the terminal
 *               snapshot (snapshots + nsteps*field, i.e. J = |u^N|^2/2); that snapshot is
 *               then overwritten.
 *   snapshots : the (nsteps+1) forward states written by dg_lserk4_fwd.
 *   eta (nullable): batch*K accumulators (caller zeroes them). */
int dg_lserk4_adj(dg_plan* plan, double* w, const double* snapshots, double t0, double dt,
                  int nsteps, double src_coef, double* eta, void* stream);

/* dg_lserk4_adj with indicator write flags (bit-identical results; fewer passes over eta):
 *   DG_ADJ_ETA_ASSIGN  the sweep's first launch assigns eta instead of adding to it, so the
 *                      caller need not zero it (nsteps = 0: eta is zeroed)
 *   DG_ADJ_ETA_ABS     the sweep's last launch stores |eta|: the per-trajectory magnitude the
 *                      reference's errorIndicator returns (python/Main_width_ref.py:139,
 *                      `return jnp.abs(err)`) before its mean over ICs (:479)
 * decisions (nullable, plans with a per-stage limiter only; ignored otherwise): the record
 * dg_lserk4_fwd_ex wrote for the same sweep.  The adjoint then takes the limiter's frozen
 * decisions from it instead of re-testing every cell, and skips the limiter work and its
 * exchange in every stage where no cell of a tile is troubled (bit-identical results). */
enum { DG_ADJ_ETA_ASSIGN = 1, DG_ADJ_ETA_ABS = 2 };
/* dg_lserk4_adj_p only: the terminal weight is P u^nsteps (J = |P u^N|^2 / 2 on the enriched
 * nodes), formed in the first launch from the snapshot it reads anyway; w's input is not read
 * (the result equals dg_prolong into w first, bit for bit). */
enum { DG_ADJ_P_TERMINAL_PROLONG = 8 };
int dg_lserk4_adj_ex(dg_plan* plan, double* w, const double* snapshots, double t0, double dt,
                     int nsteps, double src_coef, double* eta, int flags,
                     const uint16_t* decisions, void* stream);

/* Snapshot-free sweep pair (linear flux, LSERK4).  For the linear advection operator the
 * adjoint S^T does not depend on the state, and the indicator needs of each u^n only the two
 * interelement jumps per element (R = LIFT*(Fscale.*du), utils/AdvecRHS1D.m:19: du0 at the
 * left face, du1 at the right face, inflow / outflow rules as in AdvecRHS1D).  A face's jump
 * is shared by its two elements (element e's du1 = -du0 of element e+1, exactly; 0 at a
 * trajectory's last element), so the forward records one number per element and step, the
 * left-face jump, instead of the states: 8 bytes per element and step where a snapshot takes
 * 8*Np.  w, eta and the final state are bit-identical to the dg_lserk4_fwd + dg_lserk4_adj_ex
 * sweep pair with src_coef = 0 (terminal functionals, e.g. J = |u^N|^2/2 with w = u^N).
 *
 * dg_lserk4_fwd_rec: uN = u^nsteps from u0 = u^0 (u0 untouched unless uN == u0).
 *   jumps (device, 16-byte aligned, nsteps*LD doubles with LD = batch*K rounded up to even):
 *   for n = 1..nsteps and element e, jumps[(n-1)*LD + e] = du0 = u_0 - uL of u^n at t_n (uL:
 *   element e-1's u_N, or the inflow value at a trajectory's first element); the pad entry of
 *   an odd batch*K is not written.
 * dg_lserk4_adj_rec: dg_lserk4_adj_ex(w, snapshots, src_coef = 0, eta, flags) with the
 *   record of the same sweep in place of the snapshots (required whenever nsteps > 0, also
 *   without eta: DG_ERR_ARG otherwise). */
int dg_lserk4_fwd_rec(dg_plan* plan, const double* u0, double* uN, double t0, double dt,
                      int nsteps, double* jumps, void* stream);
int dg_lserk4_adj_rec(dg_plan* plan, double* w, const double* jumps, double t0, double dt,
                      int nsteps, double* eta, int flags, void* stream);

/* The whole sweep pair in one call: dg_lserk4_fwd_rec(u0 -> u^N, jumps) then
 * dg_lserk4_adj_rec(w, jumps, eta, flags) -- the reference's forward march + adjSolve + errEst
 * roles (python/Main_finite_difference.py:54-94; utils/One_code.mlx:106-140 for the march) for
 * a terminal functional.  Where the plan's record shape allows (dg_plan_query_sweep) both
 * directions run as ONE dataflow launch: the tiles of every block of steps are work items of a
 * persistent kernel that start as soon as the tiles they read have finished, so the sweep pays
 * one fill and one drain instead of one per launch.  Results are bit-identical to the two calls.
 *   u0 (in): u^0.  uN (nullable, must not alias u0 or w): receives u^nsteps.
 *   w (in/out): the terminal weight dJ/du^N on entry -- or, with DG_SWEEP_TERMINAL_STATE,
 *     u^N itself (J = |u^N|^2/2; w's content is ignored) -- and w^0 on exit.
 *   jumps: the record (layout of dg_lserk4_fwd_rec), written and read by the call.
 *   eta (nullable), flags: DG_ADJ_ETA_ASSIGN / DG_ADJ_ETA_ABS as dg_lserk4_adj_rec.
 * Scratch: the plan's (block states, indicator partials and the launch's sync words, grown on
 * the first call of a shape: make that call outside HIP-graph capture). */
enum { DG_SWEEP_TERMINAL_STATE = 4 };
int dg_lserk4_sweep_rec(dg_plan* plan, const double* u0, double* uN, double* w, double* jumps,
                        double t0, double dt, int nsteps, double* eta, int flags, void* stream);
/* dg_lserk4_sweep_rec followed by the refine decision dg_argmax_ex(eta, batch*K, use_abs = 1,
 * idx, value, nonfinite_count) -- the single-trajectory adapt iteration of
 * python/Main_finite_difference.py:336-341 (np.argmax of the indicator) up to the split.
 * In the dataflow launch the last adjoint block's tiles publish their winners and the last
 * one to arrive reduces them (no separate reduction kernels); otherwise dg_argmax_ex runs
 * after the two launch chains.  Same results either way.  eta is required; nsteps >= 1. */
int dg_lserk4_sweep_refine(dg_plan* plan, const double* u0, double* uN, double* w,
                           double* jumps, double t0, double dt, int nsteps, double* eta,
                           int flags, int64_t* idx, double* value, int64_t* nonfinite_count,
                           void* stream);
/* out[0] = 1 if dg_lserk4_sweep_rec runs nsteps as one dataflow launch (else the two launch
 * chains), out[1] / out[2] = forward / adjoint steps per block, out[3] = work items. */
int dg_plan_query_sweep(const dg_plan* plan, int nsteps, int64_t out[4]);
/* dg_plan_query_sweep plus out[4] = workgroup waves, out[5] = elements per tile. */
int dg_plan_query_sweep_ex(const dg_plan* plan, int nsteps, int64_t out[6]);
/* The dataflow launch's kernel for nsteps (profiling: what a PMC profile must match):
 * out[0] = Np, out[1] = 1 on a uniform mesh, out[2] = workgroup waves, out[3] / out[4] =
 * forward / adjoint steps per block, out[5] = elements per lane, out[6] = face exchange
 * (DG_TUNE_SWEEP_EXCHANGE), out[7] = the occupancy target in waves per SIMD (0: none).
 * out[0] = 0 when nsteps runs as the two launch chains. */
int dg_plan_query_sweep_kernel(const dg_plan* plan, int nsteps, int64_t out[8]);
/* Synchronises `stream`; *status = 0, or 1 if a dataflow sweep since the last call gave up
 * waiting for a producer (a bug, or DG_TUNE_SWEEP_SPIN_LIMIT), and clears the flag.  A work
 * item that gives up still computes, so the launch ends, but it writes NaN over its outputs
 * (states, indicator rows, its refine candidate): eta and the fused refine value are then not
 * finite and nonfinite_count counts it.  The flag is also raised in mapped host memory: every
 * later dg_lserk4_sweep_rec / dg_lserk4_sweep_refine call of the plan returns DG_ERR_HIP
 * (without a device sync) until dg_sweep_status clears it. */
int dg_sweep_status(dg_plan* plan, int* status, void* stream);
/* Profiling: with trace non-null (device), every later dataflow launch of the plan records
 * per work item the wall-clock (100 MHz) times it was taken and its producers were done and
 * it was published, and (XCC id << 32 | workgroup id): 4 uint64 per item of the jump sweep
 * (dg_plan_query_sweep's out[3] items), 8 per item of the p launches (dg_lserk4_adj_p /
 * dg_lserk4_sweep_p: dg_plan_query_p_trace).  Size it for every launch the plan runs while
 * the trace is on.  NULL turns it off.
 * HIP graphs: the dataflow launches share the plan's control words (take counter, epochs),
 * kept across launches of one shape; a dataflow call of another shape (kind, nsteps, tile,
 * waves, steps per block) re-zeroes them.  A graph that captured a dataflow launch stays
 * valid only while no call of another shape runs on the plan between its replays: re-capture
 * after one. */
int dg_plan_sweep_trace(dg_plan* plan, uint64_t* trace);

/* ---------------------------------------------------------------------------------------
 * The p-enriched dual-weighted-residual ERROR ESTIMATE.  The reference
 * marches the adjoint one order above the primal and pairs it with the primal's residual:
 * matlab/MAIN.m:32-34 (dg_march(Ns), adj_march(Ns+1)), matlab/adj_march.m:103-117
 * (err(k) = v_k'(-A uh_k - M~ + F)), python/Main_finite_difference.py:79-94 (errEst, "the
 * Adjoint-Weighted Residual as an error estimate": res[n] = u_f[n] - Phi(u_f[n-1]) of the
 * interpolated state).  Here, for the linear LSERK4 advection sweep:
 *   lo      the order-N plan of the forward sweep; hi an order-(N+1) plan on the same mesh
 *           (same K, batch, vertices, a, inflow; linear flux, no limiter, LSERK4); N <= 7
 *   P       host (N+2) x (N+1) row-major: u_hi = P u_lo, the interpolation of the element
 *           polynomials to the order-(N+1) nodes (Vandermonde1D(N, r_hi) * invV_lo)
 *   eta[e] (+)= - sum_{n=0}^{nsteps-1} w^{n+1}[e] . R^n[e],
 *           R^n = P u^{n+1} - S_{N+1}(P u^n, t_n)   (the enriched scheme's one-step residual)
 *           w^{n+1} = (S_{N+1}^T)^{nsteps-1-n} w    (the order-(N+1) discrete adjoint)
 *   so that sum_e eta[e] = w . (u_{N+1}^nsteps - P u^nsteps) with u_{N+1} the order-(N+1)
 *   march from P u^0: for a linear functional J with gradient w this is
 *   J_{N+1}(u_{N+1}) - J_{N+1}(P u_h), the DWR identity (oracle/effectivity.py p_indicator).
 *
 * dg_prolong: u_hi = P u (device fields of the lo / hi plans' sizes).
 * dg_lserk4_adj_p:
 *   w (in/out, hi field): the terminal weight dJ_{N+1}/du on entry, w^0 on exit.
 *   snapshots: the (nsteps+1) order-N states dg_lserk4_fwd wrote (snapshots[n] = u^n).
 *   eta (nullable, batch*K) and flags as dg_lserk4_adj_ex (DG_ADJ_ETA_ASSIGN / _ABS), plus
 *   DG_ADJ_P_TERMINAL_PROLONG (w on entry := P u^nsteps, formed in the kernel).
 * Scratch: the hi plan's; the dataflow form (DG_TUNE_P_FLOW) the lo plan's dataflow region
 * (as dg_lserk4_sweep_rec; its watchdog flag is the lo plan's, dg_sweep_status).  Neither plan
 * may be used concurrently. */
int dg_prolong(const dg_plan* lo, const dg_plan* hi, const double* P, const double* u,
               double* u_hi, void* stream);
int dg_lserk4_adj_p(dg_plan* lo, dg_plan* hi, const double* P, double* w,
                    const double* snapshots, double t0, double dt, int nsteps, double* eta,
                    int flags, void* stream);

/* dg_lserk4_adj_p followed by the refine decision dg_argmax_ex(lo, eta, ktot, use_abs = 1,
 * idx, value, nonfinite_count), as dg_lserk4_sweep_refine does for the jump indicator: fused
 * into the launch (the last block's tiles reduce their winners) when the estimate runs as one
 * dataflow launch (DG_TUNE_P_FLOW), else a separate reduction.  eta and idx are required.
 * Replaces python/Main_finite_difference.py:336-341 (np.argmax of the indicator). */
int dg_lserk4_adj_p_refine(dg_plan* lo, dg_plan* hi, const double* P, double* w,
                           const double* snapshots, double t0, double dt, int nsteps,
                           double* eta, int flags, int64_t* idx, double* value,
                           int64_t* nonfinite_count, void* stream);

/* *out = 1 if dg_lserk4_adj_p over nsteps steps runs as one dataflow launch on the lo plan's
 * current settings (DG_TUNE_P_FLOW, steps per launch 4, or 8 on 512-element tiles, 2..40/MS
 * blocks), else 0. */
int dg_plan_query_p_flow(const dg_plan* lo, int nsteps, int* out);

/* The p-estimate's whole sweep: the order-N LSERK4 forward from snapshot 0 (u^0, the caller's)
 * writing snapshots 1..nsteps, then dg_lserk4_adj_p with the terminal weight P u^nsteps
 * (DG_ADJ_P_TERMINAL_PROLONG implied) and, with idx non-null, the refine decision as
 * dg_lserk4_adj_p_refine.  Where the shape allows (dg_plan_query_p_sweep: the dataflow
 * estimate at 4-step blocks, the forward's workgroup tiles, 2..8 blocks) both directions run
 * as ONE dataflow launch (k_psweep: forward blocks then estimate blocks as work items), else
 * as dg_lserk4_fwd_ex at 4 steps per launch on the stage-loop workgroup tiles (whatever the
 * plan's steps per launch) + dg_lserk4_adj_p(_refine): the same bits either way, and the same
 * as dg_lserk4_fwd_ex with the lo plan's steps per launch at 4 followed by dg_lserk4_adj_p.  flags: DG_ADJ_ETA_ASSIGN /
 * _ABS.  Replaces the reference's forward march + adjoint march + error estimate
 * (matlab/MAIN.m:32-34, adj_march.m:103-117). */
int dg_lserk4_sweep_p(dg_plan* lo, dg_plan* hi, const double* P, double* snapshots, double* w,
                      double t0, double dt, int nsteps, double* eta, int flags, int64_t* idx,
                      double* value, int64_t* nonfinite_count, void* stream);

/* *out = 1 if dg_lserk4_sweep_p over nsteps steps runs as one dataflow launch, else 0. */
int dg_plan_query_p_sweep(const dg_plan* lo, int nsteps, int* out);

/* The p launches' trace records (dg_plan_sweep_trace): out[0] = work items of
 * dg_lserk4_adj_p's dataflow launch over nsteps (0: it runs as a launch chain), out[1] = work
 * items of dg_lserk4_sweep_p's (0: the chains), out[2] = uint64 words each item writes (8).  A
 * trace buffer on a plan that runs these launches needs out[2] * max(out[0], out[1]) words
 * besides the jump sweep's 4 * dg_plan_query_sweep out[3]. */
int dg_plan_query_p_trace(const dg_plan* lo, int nsteps, int64_t out[3]);

/* ulim = SlopeLimitN(u)  — utils/SlopeLimitN.m:1-33 with SlopeLimitLin.m:1-19 and minmod.m:1-13.
 * ids_mask (nullable): per element 1 if limited (the `ids` of SlopeLimitN.m:23), else 0. */
int dg_slope_limit_n(dg_plan* plan, const double* u, double* ulim, int32_t* ids_mask,
                     void* stream);

/* ulim = SlopeLimit1(u)  — utils/SlopeLimit1.m:1-23: the Pi^1 limiter (linear projection +
 * SlopeLimitLin) on every element, no troubled-cell test. */
int dg_slope_limit_1(dg_plan* plan, const double* u, double* ulim, void* stream);

/* The TVB variant of the two limiters above (the reference's optional utils/minmodB.m:6-11,
 * "the TVB modified minmod", which none of its limiters calls): with M > 0 the slope
 * SlopeLimitLin.m:18 takes is minmodB([ux; (v+ - v)/h; (v - v-)/h], M, h) -- the element's own
 * slope ux unless |ux| > M h^2, else minmod.  M = 0 (the default) is the plain minmod.  Applies
 * to dg_slope_limit_n and dg_slope_limit_1 (the per-stage limiter of the config-3 steppers
 * keeps minmod: its frozen-decision adjoint records minmod's active argument). */
int dg_plan_set_tvb(dg_plan* plan, double M);

/* idx[0] = argmax(x[0:n]) (or of |x| when use_abs), first index on ties, NaN counts as
 * maximum — numpy.argmax semantics used at python/Main_finite_difference.py:337.
 * idx is a device int64.  n <= batch*K of the plan (scratch is sized by it). */
int dg_argmax(dg_plan* plan, const double* x, int64_t n, int use_abs, int64_t* idx,
              void* stream);

/* dg_argmax plus the winning value and a non-finite count, all on the device (no host sync):
 * value (nullable device double) = x[idx] (|x[idx]| when use_abs); nonfinite_count (nullable
 * device int64) is incremented when that value is NaN or +-inf.  Under use_abs the winner is
 * non-finite exactly when some |x| is (NaN ranks first, +inf above every finite value), so a
 * count accumulated over many calls says whether any of them saw a non-finite indicator.
 * (Failure-detection role of the reference's "did not converge" messages, dg_march.m:71-73.) */
int dg_argmax_ex(dg_plan* plan, const double* x, int64_t n, int use_abs, int64_t* idx,
                 double* value, int64_t* nonfinite_count, void* stream);

/* dst[0:n] = src[0:n] with 16-byte device loads and stores (both 16-byte aligned): the
 * achievable-HBM-bandwidth ceiling of SURVEY 8(d) ("measured with a stream-copy kernel"). */
int dg_stream_copy(const double* src, double* dst, int64_t n, void* stream);

/* *device = the device address of mapped page-locked host memory `host` (e.g. a pinned
 * result buffer the refine decision is written to by dg_lserk4_sweep_refine / dg_argmax_ex
 * with no copy launch); DG_ERR_ARG if it is not such memory. */
int dg_host_alias(void* host, void** device);

/* out[k] = sum_{r=0}^{rows-1} x[r*n + k], summed in ascending r (bit-reproducible).
 * Ensemble reduction of per-IC indicators (python/Main_width_ref.py:479 mean-over-ICs role). */
int dg_sum_rows(const double* x, int64_t rows, int64_t n, double* out, void* stream);

/* One rank's refine candidate in a multi-rank ensemble (python/Main_width_ref.py:479,491: the
 * argmax of the mean indicator's magnitude, computed slice by slice): the mean
 * m[k] = (sum_{r=0}^{rows-1} x[r*ld + k]) / divisor for k < n (rows summed in ascending r,
 * as dg_sum_rows; divisor 1 skips the division, which would be exact), then i = argmax |m|
 * under numpy's order, written as cand[0] = the bits of |m[i]| (a double) and
 * cand[1] = i + offset (device int64[2]).  n <= batch*K*Np of the plan. */
int dg_slice_candidate(dg_plan* plan, const double* x, int64_t rows, int64_t n, int64_t ld,
                       double divisor, int64_t offset, int64_t* cand, void* stream);

/* The refine decision from the ranks' candidates (cands: device int64[w][2] in rank order, as
 * dg_slice_candidate writes them): the winner is the argmax of the values under numpy's
 * order (NaN first, ties to the lowest rank); idx[0] = its index, value[0] (nullable) = its
 * value, nonfinite_count[0] (nullable) += 1 when that value is not finite -- dg_argmax_ex's
 * outputs for the whole vector, bit for bit. */
int dg_candidates_argmax(const int64_t* cands, int64_t w, int64_t* idx, double* value,
                         int64_t* nonfinite_count, void* stream);

/* Synthetic ensemble initial conditions u_b(x) = amp[b] * sin(2*pi*freq[b]*x + phase[b])
 * on the plan's mesh (amp/freq/phase: device arrays of length batch). */
int dg_init_sine(const dg_plan* plan, const double* amp, const double* freq,
                 const double* phase, double* u, void* stream);

/* ---------------------------------------------------------------------------------------
 * DG-in-time marches for ensembles of the scalar ODE du/dt = sin(u).
 * Replaces matlab/dg_march.m (nonlinear branch, :36-77), matlab/adj_march.m (nonlinear
 * branch, :61-119) and the fem_setup.m operators they rebuild per slab; one ensemble member
 * (initial value y0[ic]) per lane, all members on the same slab mesh `times` (n_slabs+1
 * host-computed device doubles).  Reference-element operators are computed on the host
 * (adjoint-ode-adaptivity_amd/dgtime.py) and passed as device arrays, row-major.
 * --------------------------------------------------------------------------------------- */

/* Forward march, order Np-1, Newton per slab until ||U_old - U_next|| <= tol or maxit
 * (dg_march.m:44-68).  S = (V V')\Dr [Np][Np]; Phi [nq][Np] nodal basis at the nq Gauss
 * points (fem_setup.m:30-38); wq [nq] Gauss weights.  Y[(k*Np + i)*n_ics + ic] receives the
 * nodal values of slab k; iters (nullable) [k*n_ics + ic] the Newton iteration counts. */
int dg_time_march(int Np, int nq, const double* S, const double* Phi, const double* wq,
                  int n_slabs, const double* times, int64_t n_ics, const double* y0, double tol,
                  int maxit, double* Y, int32_t* iters, void* stream);

/* Adjoint march (order Np_fwd) for J = integral of u and the dual-weighted residual
 * err(k) = v_k' R_k(u_h) of the forward solution Y (order Np_fwd-1) (adj_march.m:66-117),
 * with the reference's slab mapping hk = x(1) - x(end) (adj_march.m:73).  Sa = inv(V V')*Dr
 * and Ma = inv(V V') [Na][Na] (Na = Np_fwd+1); Phia [nq][Na] adjoint basis at the Gauss
 * points; Pext [nq][Np_fwd] forward basis at the points adj_march.m:79 evaluates;
 * Ifa [Na][Np_fwd] forward basis at the adjoint nodes; wq [nq].  V[(k*Na + i)*n_ics + ic],
 * err[ic*n_slabs + k]. */
int dg_time_adjoint(int Np_fwd, int nq, const double* Sa, const double* Ma, const double* Phia,
                    const double* Pext, const double* Ifa, const double* wq, int n_slabs,
                    const double* times, int64_t n_ics, const double* y0, const double* Y,
                    double* V, double* err, void* stream);

/* Finite-difference DWR adapt sweep for ensembles of du/dt = sin(u), J = int u^2
 * (python/Main_finite_difference.py:34-94 and :270-277), one member (initial
 * value u0[ic]) per lane: forward Euler on the n_steps coarse steps dt_n, the discrete
 * adjoint on the ref_factor-refined grid (the bidiagonal (J_F^T - I) v = -K of :73 as its
 * backward recursion), the adjoint-weighted residual and its per-step window sums.
 * t_coarse [n_steps+1] and t_fine [n_steps*ref_factor+1] are the cumulative times of
 * interpU (:27-28); interp_code [n_steps*ref_factor+1] says where np.interp takes each fine
 * value (j >= 0: interval j; -(j+1): node j exactly).  Outputs: U[n*n_ics + ic] (coarse
 * solution), V (nullable) [n*n_ics + ic] (fine adjoint), err_steps[ic*n_steps + r]. */
int dg_fd_adapt_sweep(int n_steps, int ref_factor, const double* dt_n, const double* t_coarse,
                      const double* t_fine, const int32_t* interp_code, const double* u0,
                      int64_t n_ics, double* U, double* V, double* err_steps, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DG_ADVEC_H */
