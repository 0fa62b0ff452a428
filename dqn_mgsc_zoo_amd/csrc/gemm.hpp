// gemm.hpp — LDS-staged implicit-GEMM tile engine on gfx950 f32 MFMA.
//
// C[m][n] = sum_k A(m,k) * B(k,n), where A and B are *functors* supplied by an
// "op" (im2col of an NHWC activation, a transposed weight view, ...), so the
// conv2/conv3/fc1 layers of the NatureQNetwork forward and backward are one
// instantiation each.  The MFMA is v_mfma_f32_16x16x4_f32: exact f32 (a
// k-ordered fmaf chain, MI355X_MICROARCH.md "Matrix cores"), which is what the
// 1e-4 parity bar of BASELINE.json north_star needs.
//
// One workgroup = 256 threads = 4 waves laid out WM x WN; each wave owns
// TM x TN 16x16 accumulator tiles.  A K-stage of BK is gathered with 16-byte
// loads along each operand's contiguous axis (op::kAFastK / kBFastK), staged
// in registers one stage ahead, and written to a double-buffered LDS image
// laid out [k][m] / [k][n] with a row stride of 16 mod 32 floats (the two
// 16-lane k-groups of a 32-lane half then hit disjoint banks on the
// ds_read_b32 fragment reads).  One barrier per stage.
//
// An op provides:
//   int tiles() const; __device__ void tile_coords(int t, TileCoord&) const;
//   __device__ float4 a4(tc, m, k) const   4 elements along A's fast axis
//   __device__ float4 b4(tc, k, n) const   4 elements along B's fast axis
//   __device__ void store(tc, m, n, v) const
//   static constexpr bool kAFastK, kBFastK
// a4/b4 are called with clamped in-bounds quad origins and must not branch
// around their loads (see load_stage).
#pragma once
#include <hip/hip_runtime.h>

namespace dqz {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct TileCoord {
  int z;       // problem instance (network copy, conv phase)
  int split;   // split-K index
  int m0, n0;  // tile origin
  int k0, k1;  // K range of this split [k0, k1)
  int M, N;    // bounds of this problem
};

template <int BM_, int BN_, int BK_, int WM_, int WN_, int P_ = 3>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_, P = P_;
  static_assert(P >= 1, "prefetch depth");
  static constexpr int NT = 256;
  static_assert(WM * WN == 4, "4 waves");
  static constexpr int TM = BM / (WM * 16);
  static constexpr int TN = BN / (WN * 16);
  static_assert(TM >= 1 && TN >= 1, "tile too small");
  static_assert(BM % 32 == 0 && BN % 32 == 0 && BK % 4 == 0, "alignment");
  static constexpr int QA = BM * BK / 4 / NT;  // float4 quads per thread per stage
  static constexpr int QB = BN * BK / 4 / NT;
  static_assert(QA >= 1 && QB >= 1 && (BM * BK / 4) % NT == 0 && (BN * BK / 4) % NT == 0, "stage split");
  static constexpr int LDA = BM + 16;  // 16 mod 32 floats
  static constexpr int LDB = BN + 16;
  static constexpr int BUF = BK * (LDA + LDB);
  static constexpr int SMEM_FLOATS = 2 * BUF;
};

struct TileGrid {
  int Z, S, MT, NT_;
  __host__ __device__ int count() const { return Z * S * MT * NT_; }
  __device__ void decode(int t, int& z, int& s, int& tm, int& tn) const {
    tn = t % NT_;
    t /= NT_;
    tm = t % MT;
    t /= MT;
    s = t % S;
    z = t / S;
  }
};

// (m, k) origin of quad q of an operand whose fast axis is k (FastK) or m.
template <int ROWS, int BK, bool FastK>
__device__ __forceinline__ void quad_pos(int q, int& r, int& k) {
  if constexpr (FastK) {
    k = (q % (BK / 4)) * 4;
    r = q / (BK / 4);
  } else {
    r = (q % (ROWS / 4)) * 4;
    k = q / (ROWS / 4);
  }
}

// Branch-free stage gather: every quad issues exactly one 16-byte load from a
// clamped (always in-bounds) coordinate and out-of-range elements are zeroed
// by selects afterwards.  A bounds check *around* a load makes hipcc drain
// every outstanding load (s_waitcnt vmcnt(0)) at each use, which serialises
// the prefetch ring (cdna_hip_programming.md §5, "Three .s-level traps" (c)).
// Contract: a FastK operand has K % 4 == 0 inside every split, so a k-quad is
// either fully in or fully out of [k0, k1); along m/n a quad may straddle
// M/N and the op must return in-bounds memory for its first element.
template <class C>
struct StageRegs {
  float4 a[C::QA];
  float4 b[C::QB];
  unsigned ma, mb;  // 4 validity bits per quad; applied when written to LDS
};

template <class C, class Op>
__device__ __forceinline__ void load_stage(const Op& op, const TileCoord& tc, int kt, StageRegs<C>& r) {
  const int t = threadIdx.x;
  r.ma = 0;
  r.mb = 0;
#pragma unroll
  for (int e = 0; e < C::QA; ++e) {
    int m, k;
    quad_pos<C::BM, C::BK, Op::kAFastK>(t + e * C::NT, m, k);
    const int gm = tc.m0 + m, gk = kt + k;
    const bool kin = gk < tc.k1;
    r.a[e] = op.a4(tc, gm < tc.M ? gm : tc.m0, kin ? gk : tc.k0);
    unsigned bits;
    if constexpr (Op::kAFastK) {
      bits = (kin && gm < tc.M) ? 0xFu : 0u;
    } else {
      const int live = kin ? min(4, max(0, tc.M - gm)) : 0;
      bits = (1u << live) - 1u;
    }
    r.ma |= bits << (4 * e);
  }
#pragma unroll
  for (int e = 0; e < C::QB; ++e) {
    int n, k;
    quad_pos<C::BN, C::BK, Op::kBFastK>(t + e * C::NT, n, k);
    const int gn = tc.n0 + n, gk = kt + k;
    const bool kin = gk < tc.k1;
    r.b[e] = op.b4(tc, kin ? gk : tc.k0, gn < tc.N ? gn : tc.n0);
    unsigned bits;
    if constexpr (Op::kBFastK) {
      bits = (kin && gn < tc.N) ? 0xFu : 0u;
    } else {
      const int live = kin ? min(4, max(0, tc.N - gn)) : 0;
      bits = (1u << live) - 1u;
    }
    r.mb |= bits << (4 * e);
  }
}

__device__ __forceinline__ float4 masked(float4 v, unsigned bits) {
  v.x = (bits & 1u) ? v.x : 0.f;
  v.y = (bits & 2u) ? v.y : 0.f;
  v.z = (bits & 4u) ? v.z : 0.f;
  v.w = (bits & 8u) ? v.w : 0.f;
  return v;
}

template <class C, class Op>
__device__ __forceinline__ void store_stage(float* As, float* Bs, const StageRegs<C>& r) {
  const int t = threadIdx.x;
#pragma unroll
  for (int e = 0; e < C::QA; ++e) {
    int m, k;
    quad_pos<C::BM, C::BK, Op::kAFastK>(t + e * C::NT, m, k);
    const float4 v = masked(r.a[e], r.ma >> (4 * e));
    if constexpr (Op::kAFastK) {
      As[(k + 0) * C::LDA + m] = v.x;
      As[(k + 1) * C::LDA + m] = v.y;
      As[(k + 2) * C::LDA + m] = v.z;
      As[(k + 3) * C::LDA + m] = v.w;
    } else {
      *reinterpret_cast<float4*>(&As[k * C::LDA + m]) = v;
    }
  }
#pragma unroll
  for (int e = 0; e < C::QB; ++e) {
    int n, k;
    quad_pos<C::BN, C::BK, Op::kBFastK>(t + e * C::NT, n, k);
    const float4 v = masked(r.b[e], r.mb >> (4 * e));
    if constexpr (Op::kBFastK) {
      Bs[(k + 0) * C::LDB + n] = v.x;
      Bs[(k + 1) * C::LDB + n] = v.y;
      Bs[(k + 2) * C::LDB + n] = v.z;
      Bs[(k + 3) * C::LDB + n] = v.w;
    } else {
      *reinterpret_cast<float4*>(&Bs[k * C::LDB + n]) = v;
    }
  }
}

// Runs one output tile of `op` (all of its K range) on the calling workgroup.
// Register ring of C::P stages: stage t is issued P compute phases before it
// is written to LDS, so P stages of global-load latency hide behind MFMAs.
template <class C, class Op>
__device__ void gemm_tile(const Op& op, const TileCoord& tc, float* smem) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int fr = lane & 15, fk = lane >> 4;

  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Loads are unconditional (stages past the end are masked to zero), so
  // hipcc's waitcnt pass sees the same load stream on every path and keeps
  // P stages in flight; only the LDS-only compute is guarded.
  StageRegs<C> ring[C::P];
  const int nstage = (tc.k1 - tc.k0 + C::BK - 1) / C::BK;
#pragma unroll
  for (int j = 0; j < C::P; ++j) load_stage<C>(op, tc, tc.k0 + j * C::BK, ring[j]);
  store_stage<C, Op>(smem, smem + C::BK * C::LDA, ring[0]);
  load_stage<C>(op, tc, tc.k0 + C::P * C::BK, ring[0]);
  __syncthreads();
  for (int s0 = 0; s0 < nstage; s0 += C::P) {
#pragma unroll
    for (int j = 0; j < C::P; ++j) {
      const int s = s0 + j;
      if (s < nstage) {
        const float* As = smem + (s & 1) * C::BUF;
        const float* Bs = As + C::BK * C::LDA;
        // All fragments of the stage are read before the first MFMA: at one
        // wave per SIMD nothing else hides a ds_read -> MFMA dependency.
        constexpr int KS = C::BK / 4;
        float av[KS][C::TM], bv[KS][C::TN];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
          for (int i = 0; i < C::TM; ++i) av[kk][i] = As[(4 * kk + fk) * C::LDA + (wm * C::TM + i) * 16 + fr];
#pragma unroll
          for (int q = 0; q < C::TN; ++q) bv[kk][q] = Bs[(4 * kk + fk) * C::LDB + (wn * C::TN + q) * 16 + fr];
        }
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int i = 0; i < C::TM; ++i)
#pragma unroll
            for (int q = 0; q < C::TN; ++q)
              acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk][i], bv[kk][q], acc[i][q], 0, 0, 0);
      }
      const int nx = (j + 1) % C::P;  // ring slot holding stage s + 1 (static after unroll)
      float* An = smem + ((s + 1) & 1) * C::BUF;
      store_stage<C, Op>(An, An + C::BK * C::LDA, ring[nx]);
      load_stage<C>(op, tc, tc.k0 + (s + 1 + C::P) * C::BK, ring[nx]);
      __syncthreads();
    }
  }
  // Epilogue: C/D map of 16x16x4 f32: col = lane & 15, row = (lane >> 4) * 4 + r.
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = tc.m0 + (wm * C::TM + i) * 16 + fk * 4 + r;
        const int n = tc.n0 + (wn * C::TN + j) * 16 + fr;
        if (m < tc.M && n < tc.N) op.store(tc, m, n, acc[i][j][r]);
      }
}

// Placeholder op for unused slots of a multi-op launch.
struct NoOp {
  static constexpr bool kAFastK = true, kBFastK = false;
  __host__ __device__ int tiles() const { return 0; }
  __device__ void tile_coords(int, TileCoord&) const {}
  __device__ float4 a4(const TileCoord&, int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ float4 b4(const TileCoord&, int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void store(const TileCoord&, int, int, float) const {}
};

// One launch runs the tiles of up to three independent ops (e.g. conv dX and
// conv dW of the same layer, which only share their inputs): tile ids
// [0, n1) -> op1, [n1, n1+n2) -> op2, rest -> op3.
template <class C, class Op1, class Op2, class Op3>
__global__ __launch_bounds__(256) void multi_gemm_kernel(Op1 op1, Op2 op2, Op3 op3, int n1, int n2) {
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_FLOATS];
  int t = blockIdx.x;
  TileCoord tc;
  if (t < n1) {
    op1.tile_coords(t, tc);
    gemm_tile<C>(op1, tc, smem);
  } else if (t < n1 + n2) {
    op2.tile_coords(t - n1, tc);
    gemm_tile<C>(op2, tc, smem);
  } else {
    op3.tile_coords(t - n1 - n2, tc);
    gemm_tile<C>(op3, tc, smem);
  }
}

template <class C, class Op1, class Op2 = NoOp, class Op3 = NoOp>
inline hipError_t launch_gemm(hipStream_t s, const Op1& op1, const Op2& op2 = Op2(), const Op3& op3 = Op3()) {
  const int n1 = op1.tiles(), n2 = op2.tiles(), n3 = op3.tiles();
  const int total = n1 + n2 + n3;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL((multi_gemm_kernel<C, Op1, Op2, Op3>), dim3(total), dim3(256), 0, s, op1, op2, op3, n1, n2);
  return hipGetLastError();
}

// Shape shared by the ops: tile grid + problem bounds + split-K length.
struct Shape {
  TileGrid g;
  int M, N, K, KS, BM, BN;
  __device__ __forceinline__ void coords(int t, TileCoord& tc) const {
    int z, s, tm, tn;
    g.decode(t, z, s, tm, tn);
    tc.z = z;
    tc.split = s;
    tc.m0 = tm * BM;
    tc.n0 = tn * BN;
    tc.k0 = s * KS;
    tc.k1 = min(K, (s + 1) * KS);
    tc.M = M;
    tc.N = N;
  }
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __host__ __device__ int tiles() const { return g.count(); }
};

template <class C>
inline Shape make_shape(int Z, int M, int N, int K, int S) {
  Shape sh;
  int ks = (K + S - 1) / S;
  ks = (ks + C::BK - 1) / C::BK * C::BK;
  S = (K + ks - 1) / ks;
  sh.g.Z = Z;
  sh.g.S = S;
  sh.g.MT = (M + C::BM - 1) / C::BM;
  sh.g.NT_ = (N + C::BN - 1) / C::BN;
  sh.M = M;
  sh.N = N;
  sh.K = K;
  sh.KS = ks;
  sh.BM = C::BM;
  sh.BN = C::BN;
  return sh;
}

}  // namespace dqz
