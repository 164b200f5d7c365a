// wave_hip.h — the gfx950 wave policy (W) for the engine templates: one 64-lane wavefront per env.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct WaveHip {
  static constexpr int kWidth = 64;
  // SSIM_OPAQUE_LANE (set per translation unit, for the 4-wave HBM-resident kernels): the lane index behind an empty
  // asm at every use. From a plain __lane_id() the compiler hoists every per-lane address and lane condition derived
  // from it (base + lane x stride, for dozens of arrays) to the kernel entry, where at the 128-VGPR cap they are spilled
  // to scratch memory and reloaded at each use; opaque, each is recomputed (a VALU op or two) where it is used.
#if SSIM_OPAQUE_LANE
  __device__ static __forceinline__ int lane() {
    int l = (int)__lane_id();
    asm volatile("" : "+v"(l));
    return l;
  }
#else
  __device__ static __forceinline__ int lane() { return (int)__lane_id(); }
#endif
  __device__ static __forceinline__ uint64_t ballot(bool p) { return (uint64_t)__ballot(p); }
  __device__ static __forceinline__ int ffs(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }
  __device__ static __forceinline__ int popc(uint64_t m) { return __popcll((unsigned long long)m); }
  __device__ static __forceinline__ int rank(uint64_t m) {  // set bits of m below this lane
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  }
  // Wave-uniform value -> SGPR. The serial part of the algorithm runs on values every lane holds
  // identically; v_readfirstlane makes that provable, so its arithmetic is SALU and its branches are
  // s_cbranch_scc instead of exec-mask (divergent) control flow.
  __device__ static __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
  __device__ static __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
  __device__ static __forceinline__ int16_t uni(int16_t v) { return (int16_t)__builtin_amdgcn_readfirstlane((int)v); }
  __device__ static __forceinline__ uint16_t uni(uint16_t v) { return (uint16_t)__builtin_amdgcn_readfirstlane((int)v); }
  __device__ static __forceinline__ uint8_t uni(uint8_t v) { return (uint8_t)__builtin_amdgcn_readfirstlane((int)v); }
  __device__ static __forceinline__ int8_t uni(int8_t v) { return (int8_t)__builtin_amdgcn_readfirstlane((int)v); }
  __device__ static __forceinline__ uint64_t uni(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
  }
  __device__ static __forceinline__ int64_t uni(int64_t v) { return (int64_t)uni((uint64_t)v); }
  __device__ static __forceinline__ float uni(float v) {
    return __builtin_bit_cast(float, uni(__builtin_bit_cast(uint32_t, v)));
  }
  template <class T>
  __device__ static __forceinline__ T* uni(T* p) {
    return reinterpret_cast<T*>(uni(reinterpret_cast<uint64_t>(p)));
  }
  __device__ static __forceinline__ double uni(double v) {
    return __builtin_bit_cast(double, uni(__builtin_bit_cast(uint64_t, v)));
  }
  // v_readlane (VALU -> SGPR) instead of an LDS-path ds_bpermute; `l` is wave-uniform
  __device__ static __forceinline__ int bcast_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
  __device__ static __forceinline__ double bcast_d(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
  }
  __device__ static __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // Drains every outstanding memory operation of the wave (s_waitcnt 0). Lane-parallel scratch traffic whose stores,
  // atomics and loads may be issued as different instruction kinds (FLAT through the texture path, DS direct to the
  // LDS: not ordered against each other) is fenced with it before the data is read back.
  __device__ static __forceinline__ void drain() {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
  __device__ static __forceinline__ void gsync() {  // global-memory ordering across the wave's lanes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  __device__ static __forceinline__ uint64_t clock() { return __builtin_amdgcn_s_memtime(); }
  __device__ static __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz
  // no-return LDS atomic add (diagnostic profile build)
  __device__ static __forceinline__ void lds_add_u64(uint64_t* p, uint64_t v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  // Cross-lane reads through ds_bpermute with the source lane computed from lane() (opaque in the 4-wave units): HIP's
  // __shfl_xor / __shfl_up compute it from their own __lane_id(), and the compiler hoisted those per-lane addresses
  // (six per butterfly) to the kernel entry and spilled them.
  __device__ static __forceinline__ int shfl_xor_i(int v, int off) {
    return __builtin_amdgcn_ds_bpermute((lane() ^ off) << 2, v);
  }
  __device__ static __forceinline__ float shfl_xor_f(float v, int off) {
    return __builtin_bit_cast(float, shfl_xor_i(__builtin_bit_cast(int, v), off));
  }
  __device__ static __forceinline__ double shfl_xor_d(double v, int off) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int a = (lane() ^ off) << 2;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
  }
  __device__ static __forceinline__ int excl_scan(int x, int* total) {
    int v = x;
    const int l = lane();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __builtin_amdgcn_ds_bpermute(((l - off) & 63) << 2, v);  // (used only where l >= off)
      if (l >= off) v += y;
    }
    *total = __builtin_amdgcn_readlane(v, 63);  // SGPR: the running total stays wave-uniform
    return v - x;
  }
  __device__ static __forceinline__ double sum_d(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += shfl_xor_d(x, off);
    return uni(x);
  }
  // Sparse argmins: the candidates are few (live commitments, pending executor events), so walk the
  // ballot of valid lanes with v_readlane instead of a 6-round ds_bpermute butterfly.
  // lexicographic min of (key, val) over lanes with key != INT_MAX; result in every lane (SGPRs: the
  // accumulators start from constants, never from a lane's own value, so they stay wave-uniform).
  // With no candidate, key = INT_MAX and val = -1.
  __device__ static __forceinline__ void min_pair(int& key, int& val) {
    uint64_t m = ballot(key != 0x7FFFFFFF);
    int bk = 0x7FFFFFFF, bv = -1;
    while (m) {
      const int l = ffs(m);
      m &= m - 1;
      const int k2 = bcast_i(key, l), v2 = bcast_i(val, l);
      if (k2 < bk || (k2 == bk && v2 < bv)) {
        bk = k2;
        bv = v2;
      }
    }
    key = bk;
    val = bv;
  }
  // Wave min of a double over lanes [0, kSpan) (kSpan 16 or 64), wave-uniform result. Row stages are DPP
  // (quad xor 1, xor 2, row_ror 4, row_ror 8: every lane of a row ends with the row min), then for a full
  // wave the four row minima are combined on the scalar side. All 64 lanes must be active (callers run in
  // wave-uniform control flow).
  template <int kCtrl>
  __device__ static __forceinline__ uint64_t dpp_u(uint64_t b) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, kCtrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), kCtrl, 0xF, 0xF, false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
  }
  __device__ static __forceinline__ uint64_t umin(uint64_t a, uint64_t b) { return b < a ? b : a; }
  // Event times are non-negative doubles or +inf, whose bit patterns order like unsigned integers: the min runs on
  // the bits (no canonicalising f64 min).
  template <int kSpan>
  __device__ static __forceinline__ double min_d(double v) {
    uint64_t b = __builtin_bit_cast(uint64_t, v);
    b = umin(b, dpp_u<0xB1>(b));   // quad_perm [1,0,3,2]
    b = umin(b, dpp_u<0x4E>(b));   // quad_perm [2,3,0,1]
    b = umin(b, dpp_u<0x124>(b));  // row_ror:4
    b = umin(b, dpp_u<0x128>(b));  // row_ror:8
    uint64_t m = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 0) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 0) << 32);
    if (kSpan > 16) {
      for (int r = 16; r < 64; r += 16) {
        const uint64_t mr = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, r) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), r) << 32);
        m = umin(m, mr);
      }
      m = uni(m);
    }
    return __builtin_bit_cast(double, m);
  }
  // Argmin of (t, seq) over lanes [0, kSpan) with `valid`: the winning lane (-1 if none). One DPP min of t,
  // then the (rare) ties on t are broken by the smaller seq. `tmin` receives the winning t.
  template <int kSpan>
  __device__ static __forceinline__ int argmin_event(double t, int seq, bool valid, double* tmin) {
    const double m = min_d<kSpan>(valid ? t : __builtin_inf());
    uint64_t eq = ballot(valid && t == m);
    *tmin = m;
    if (eq == 0) return -1;
    int l = ffs(eq);
    eq &= eq - 1;
    if (eq) {
      int bs = bcast_i(seq, l);
      while (eq) {
        const int l2 = ffs(eq);
        eq &= eq - 1;
        const int s2 = bcast_i(seq, l2);
        if (s2 < bs) {
          bs = s2;
          l = l2;
        }
      }
    }
    return l;
  }
  // wave-uniform value into lane `l` of a per-lane value (`l` wave-uniform)
  __device__ static __forceinline__ int writelane(int v, int l, int old) { return lane() == l ? v : old; }
  // Forward permute: this lane's v goes to lane `dst` (a permutation of the lanes; ds_permute_b32)
  __device__ static __forceinline__ int permute_to(int dst, int v) { return __builtin_amdgcn_ds_permute(dst << 2, v); }
  // Compaction keeping lane order: lanes in `m` move to lanes 0..popc(m)-1, the rest after them
  __device__ static __forceinline__ int compact(uint64_t m, int v) {
    const bool in = (m >> lane()) & 1ull;
    return permute_to(in ? rank(m) : popc(m) + rank(~m), v);
  }
  // correctly rounded f32 ops (the reference's numpy float32 arithmetic; no contraction)
  __device__ static __forceinline__ float fdiv(float a, float b) { return __fdiv_rn(a, b); }
  __device__ static __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
  // streaming (non-temporal) global store
  template <class T>
  __device__ static __forceinline__ void st_nt(T* p, T v) { __builtin_nontemporal_store(v, p); }
  // Atomics / loads for lane-parallel relaxations over LDS or a wave's own global scratch: workgroup scope (the data
  // is private to the wave). On global memory the atomics are performed in L2 and the load carries sc0 (it bypasses
  // the CU's L1), so it sees them; system / agent scope would take the atomics to memory and make fences write back
  // and invalidate the L2.
  __device__ static __forceinline__ int lds_load(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ static __forceinline__ float ld_rel(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ static __forceinline__ void amax(int* p, int v) {
    __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ static __forceinline__ void amin(int* p, int v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ static __forceinline__ void aor(uint32_t* p, uint32_t v) {
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ static __forceinline__ void fadd(float* p, float v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ static __forceinline__ float max_f(float x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float y = shfl_xor_f(x, off);
      x = y > x ? y : x;
    }
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
  }
  __device__ static __forceinline__ float sum_f(float x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += shfl_xor_f(x, off);
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
  }
  __device__ static __forceinline__ int min_i(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const int y = shfl_xor_i(x, off);
      x = y < x ? y : x;
    }
    return uni(x);
  }
  __device__ static __forceinline__ int max_i(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const int y = shfl_xor_i(x, off);
      x = y > x ? y : x;
    }
    return uni(x);
  }
};
