// dg_flow.h — the dataflow launches' shared device primitives: the control-word layout, the
// flag poll with its watchdog, and the give-up poisoning.  Used by the jump-record sweep
// (dg_sweep_kernel.h, k_sweep_rp) and the p-enriched estimate's one-launch sweep (dg_dwr.hip,
// k_adjp_flow).  The hand-off protocol they implement is described in dg_sweep_kernel.h.
// Internal to libdgadv.so.
#pragma once
#include "dg_rec_tiles.h"

namespace dgr {

constexpr int kSweepMaxSteps = 40;   // steps per dataflow launch (block constants are kernargs)
constexpr int kSweepMaxBlocks = 8;   // jump sweep: blocks per direction (kSweepMaxSteps / 5)
// control words (uint32 index): a 64-bit take counter, the error word, a 64-bit arrival
// counter of the fused refine decision, then one flag per item
constexpr int kSyncHead = 0, kSyncErr = 2, kSyncArrive = 4, kSyncFlags = 16;
constexpr int kSweepSpinLimit = 1 << 20;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st8_agent(void* p, uint64_t bits) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), bits, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld8_agent(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Thread 0: take the next item of a launch of `nItems` items from the 64-bit take counter.
// The counter only grows: every launch of one shape takes exactly nItems values (one per
// workgroup), so h / nItems numbers the launch (its epoch - 1) and h % nItems is the item --
// no reset, no generation word, no exit counter.  (The host zeroes the control words when a
// launch of another shape reuses them.)  Items start in queue order whatever order the
// dispatcher starts workgroups in: the dataflow launches' deadlock-freedom rests on that alone.
__device__ __forceinline__ void flow_take(uint32_t* sync, int64_t nItems, uint32_t* item,
                                          uint32_t* epoch) {
  const uint64_t h = __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(sync + kSyncHead),
                                            uint64_t(1), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
  *epoch = uint32_t(h / uint64_t(nItems)) + 1u;
  *item = uint32_t(h % uint64_t(nItems));
}

// Wave 0: wait until flags[0..nd) all hold `epoch` (one lane per flag, nd <= 64).  Returns
// true (wave-uniform) if it gave up: after `limit` polls (a producer that never finishes; the
// launch's error word and the host-visible flag are raised) or on seeing the error word.
__device__ __forceinline__ bool sweep_wait(const uint32_t* flags, int nd, uint32_t epoch,
                                           uint32_t* sync, uint32_t* err_host, int limit) {
  const int l = threadIdx.x & 63;
  bool ok = l >= nd;
  if (!ok) ok = ld_agent(flags + l) == epoch;
  int spins = 0;
  while (!__all(ok)) {
    __builtin_amdgcn_s_sleep(2);
    if (!ok) ok = ld_agent(flags + l) == epoch;
    if (++spins >= limit) {
      if (l == 0) {
        st_agent(sync + kSyncErr, 1u);
        if (err_host)
          __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return true;
    }
    if ((spins & 255) == 0 && ld_agent(sync + kSyncErr) != 0u) return true;  // someone gave up
  }
  return false;
}

// A work item that gave up computed on inputs that may not have been ready: it overwrites
// what it publishes with NaN (write-through, like the outputs), so every consumer, the
// indicator and the fused refine decision turn non-finite and the callers' checks fire.
template <int LB>
__device__ __forceinline__ void poison_run(double* __restrict__ g, int64_t o0, int64_t count) {
  if (count <= 0) return;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(g + o0);
  const double q = __builtin_nan("");
  for (int64_t v = threadIdx.x; v < count; v += LB) wt_st8(r, uint32_t(v) * 8u, q);
}

// Winner of (v, i) over the NW-wave workgroup under am_better; valid in thread 0.  sv / si:
// NW LDS slots of the caller's own (not aliased with a tile image another wave may read).
template <int NW>
__device__ __forceinline__ void wg_argmax(double& v, int64_t& i, double* sv, int64_t* si) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const int64_t oi = __shfl_xor(i, off);
    if (am_better(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[wv] = v;
    si[wv] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k < NW; ++k)
      if (am_better(sv[k], si[k], v, i)) {
        v = sv[k];
        i = si[k];
      }
}

// The fused refine decision's last step (thread 0 of every workgroup of the last block, after
// its tile's winner was published write-through and drained): the tiles arrive on a counter
// that grows by nT per launch; the one whose add completes a launch's count reduces the nT
// winners with agent-scope loads and writes dg_argmax_ex's outputs.  Call from all threads.
template <int NW>
__device__ __forceinline__ void flow_refine_arrive(uint32_t* sync, int nT, const double* pv,
                                                   const int64_t* pi, int64_t* am_idx,
                                                   double* am_val, int64_t* am_nf,
                                                   uint32_t* s_last, double* s_av,
                                                   int64_t* s_ai) {
  if (threadIdx.x == 0) {
    const uint64_t old = __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(sync + kSyncArrive),
                                                uint64_t(1), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    *s_last = ((old + 1) % uint64_t(nT)) == 0 ? 1u : 0u;
  }
  __syncthreads();
  if (*s_last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double v = -INFINITY;
    int64_t i = INT64_MAX;
    for (int q = threadIdx.x; q < nT; q += 64 * NW) {
      const double qv = __builtin_bit_cast(double, ld8_agent(pv + q));
      const int64_t qi = int64_t(ld8_agent(pi + q));
      if (am_better(qv, qi, v, i)) {
        v = qv;
        i = qi;
      }
    }
    wg_argmax<NW>(v, i, s_av, s_ai);
    if (threadIdx.x == 0) {
      if (ld_agent(sync + kSyncErr) != 0u) v = __builtin_nan("");  // a work item gave up
      am_idx[0] = i;
      if (am_val) am_val[0] = v;
      if (am_nf && !isfinite(v)) am_nf[0] += 1;
    }
  }
}

}  // namespace dgr
