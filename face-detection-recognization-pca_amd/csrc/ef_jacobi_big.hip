// Symmetric eigensolver for orders beyond the LDS Jacobi (m > kJacobiMax): the same
// cyclic two-sided Jacobi method (circle ordering, m/2 disjoint rotations per round,
// rotation skip test and sweep-level convergence of jacobi_kernel in ef_linalg.hip),
// with the matrix and the eigenvector accumulator in HBM/L2 and every round spread over
// the whole GPU:
//   * one launch per round; thread (t, u) owns the 2 x 2 block rows {p_t, q_t} x columns
//     {p_u, q_u} and applies both rotations (G' = J^T G J) — no intra-round barrier;
//   * the rotation of each pair is recomputed by every thread that needs it from the
//     round's input matrix, which is therefore ping-ponged (in-place would race on the
//     pivots); V <- V J is in place (thread (i, u) owns V[i][p_u], V[i][q_u]);
//   * a sweep whose pivots are all below 1e-12 of their diagonal scale ends the solve
//     (one host read of a flag per sweep).
// Used for the Rayleigh-Ritz / orthonormalisation problems of the subspace iteration at
// k > 80 (BASELINE.json config 3: k = 128; config 5: k = 512) and for direct solves of
// moderate orders.  Quadratic convergence: a nearly diagonal input (warm subspace) needs
// 2-3 sweeps.
#include "ef_linalg.hpp"

namespace ef {

__device__ __forceinline__ int circle_pos(int j, int r, int mp) { return j == 0 ? 0 : 1 + ((j - 1 + r) % (mp - 1)); }

struct Rot {
  int p, q;
  double c, s;
  bool on;
};

__device__ __forceinline__ Rot pair_rotation(const double* __restrict__ G, int mp, int r, int t) {
  Rot R;
  int p = circle_pos(t, r, mp), q = circle_pos(mp - 1 - t, r, mp);
  if (p > q) { const int x = p; p = q; q = x; }
  R.p = p;
  R.q = q;
  const double apq = G[(int64_t)p * mp + q];
  const double app = G[(int64_t)p * mp + p], aqq = G[(int64_t)q * mp + q];
  const double g = 100.0 * fabs(apq);
  if (apq == 0.0 || (fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq))) {
    R.on = false;
    R.c = 1.0;
    R.s = 0.0;
  } else {
    const double theta = (aqq - app) / (2.0 * apq);
    double tt = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
    if (fabs(theta) > 1e150) tt = 0.5 / fabs(theta);
    if (theta < 0.0) tt = -tt;
    R.c = 1.0 / sqrt(tt * tt + 1.0);
    R.s = tt * R.c;
    R.on = true;
  }
  return R;
}

__global__ void jbig_init_kernel(const double* __restrict__ A, int m, int64_t lda, int mp, double* __restrict__ G,
                                 double* __restrict__ V) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)mp * mp) return;
  const int i = (int)(e / mp), j = (int)(e - (e / mp) * mp);
  G[e] = (i < m && j < m) ? 0.5 * (A[(int64_t)i * lda + j] + A[(int64_t)j * lda + i]) : 0.0;
  V[e] = i == j ? 1.0 : 0.0;
}

__global__ __launch_bounds__(256) void jbig_round_kernel(const double* __restrict__ Gin, double* __restrict__ Gout,
                                                        double* __restrict__ V, int mp, int r, int* __restrict__ flag) {
  const int np = mp / 2;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)np * np;
  if (e < nb) {
    const int t = (int)(e / np), u = (int)(e - (e / np) * np);
    const Rot a = pair_rotation(Gin, mp, r, t);
    const Rot b = t == u ? a : pair_rotation(Gin, mp, r, u);
    const double x00 = Gin[(int64_t)a.p * mp + b.p], x01 = Gin[(int64_t)a.p * mp + b.q];
    const double x10 = Gin[(int64_t)a.q * mp + b.p], x11 = Gin[(int64_t)a.q * mp + b.q];
    // rows: p <- c p - s q, q <- s p + c q
    const double y00 = a.c * x00 - a.s * x10, y01 = a.c * x01 - a.s * x11;
    const double y10 = a.s * x00 + a.c * x10, y11 = a.s * x01 + a.c * x11;
    // columns, same convention
    double z00 = b.c * y00 - b.s * y01, z01 = b.s * y00 + b.c * y01;
    double z10 = b.c * y10 - b.s * y11, z11 = b.s * y10 + b.c * y11;
    if (t == u && a.on) {
      z01 = 0.0;
      z10 = 0.0;
      // a sweep whose rotated pivots were all below 1e-12 of their diagonal scale ends
      // the solve: the matrix is then diagonal to ~1e-12 relative (near-degenerate pairs
      // may still rotate by large angles without extending the sweep count)
      if (fabs(x01) > 1e-12 * sqrt(fabs(x00 * x11))) *flag = 1;
    }
    Gout[(int64_t)a.p * mp + b.p] = z00;
    Gout[(int64_t)a.p * mp + b.q] = z01;
    Gout[(int64_t)a.q * mp + b.p] = z10;
    Gout[(int64_t)a.q * mp + b.q] = z11;
    return;
  }
  const int64_t f = e - nb;
  if (f >= (int64_t)mp * np) return;
  const int i = (int)(f / np), u = (int)(f - (f / np) * np);
  const Rot b = pair_rotation(Gin, mp, r, u);
  if (!b.on) return;
  const double vp = V[(int64_t)i * mp + b.p], vq = V[(int64_t)i * mp + b.q];
  V[(int64_t)i * mp + b.p] = b.c * vp - b.s * vq;
  V[(int64_t)i * mp + b.q] = b.s * vp + b.c * vq;
}

// descending order (ties -> lower index first); evecs[r][rank] = V[r][i]
__global__ void jbig_sort_kernel(const double* __restrict__ G, const double* __restrict__ V, int m, int mp,
                                 double* __restrict__ evals, double* __restrict__ evecs, int64_t ldv) {
  const int i = blockIdx.x;
  __shared__ int rank_s;
  const double li = G[(int64_t)i * mp + i];
  if (threadIdx.x == 0) rank_s = 0;
  __syncthreads();
  int cnt = 0;
  for (int j = threadIdx.x; j < m; j += blockDim.x) {
    const double lj = G[(int64_t)j * mp + j];
    cnt += (lj > li) || (lj == li && j < i);
  }
  atomicAdd(&rank_s, cnt);
  __syncthreads();
  const int rank = rank_s;
  if (threadIdx.x == 0) evals[rank] = li;
  for (int rr = threadIdx.x; rr < m; rr += blockDim.x) evecs[(int64_t)rr * ldv + rank] = V[(int64_t)rr * mp + i];
}

size_t jacobi_big_work_elems(int m) {
  const int64_t mp = m + (m & 1);
  return (size_t)(3 * mp * mp) + 64;
}

// One sweep (mp - 1 rounds) per graph; two graphs for the two ping-pong parities.
void JacobiBig::destroy() {
  for (auto& g : exec)
    if (g) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(g));
  exec[0] = exec[1] = nullptr;
}

hipError_t JacobiBig::init(int m_, double* work_, int* flag_, hipStream_t capture) {
  destroy();
  m = m_;
  mp = m + (m & 1);
  work = work_;
  flag = flag_;
  double* G[2] = {work, work + (int64_t)mp * mp};
  double* V = work + 2 * (int64_t)mp * mp;
  const int np = mp / 2;
  const int64_t threads = (int64_t)np * np + (int64_t)mp * np;
  const dim3 grid((unsigned)((threads + 255) / 256));
  for (int par = 0; par < 2; ++par) {
    hipError_t e = hipStreamBeginCapture(capture, hipStreamCaptureModeRelaxed);
    if (e != hipSuccess) return e;
    (void)hipMemsetAsync(flag, 0, sizeof(int), capture);
    int cur = par;
    for (int r = 0; r < mp - 1; ++r) {
      hipLaunchKernelGGL(jbig_round_kernel, grid, dim3(256), 0, capture, G[cur], G[cur ^ 1], V, mp, r, flag);
      cur ^= 1;
    }
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(capture, &g);
    if (e != hipSuccess) return e;
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return e;
    exec[par] = x;
  }
  return hipSuccess;
}

int JacobiBig::solve(hipStream_t s, const double* A, int64_t lda, double* evals, double* evecs, int64_t ldv,
                     int max_sweeps, int* sweeps_out, hipError_t* err) {
  double* G[2] = {work, work + (int64_t)mp * mp};
  double* V = work + 2 * (int64_t)mp * mp;
  const int64_t tot = (int64_t)mp * mp;
  hipLaunchKernelGGL(jbig_init_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, A, m, lda, mp, G[0], V);
  int cur = 0, sweep = 0;
  bool converged = false;
  for (; sweep < max_sweeps; ++sweep) {
    *err = hipGraphLaunch(static_cast<hipGraphExec_t>(exec[cur]), s);
    if (*err != hipSuccess) return -1;
    cur ^= (mp - 1) & 1;  // an odd number of rounds swaps the buffers
    int hflag = 0;
    *err = hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s);
    if (*err == hipSuccess) *err = hipStreamSynchronize(s);
    if (*err != hipSuccess) return -1;
    if (hflag == 0) {
      converged = true;
      break;
    }
  }
  hipLaunchKernelGGL(jbig_sort_kernel, dim3((unsigned)m), dim3(256), 0, s, G[cur], V, m, mp, evals, evecs, ldv);
  *err = hipGetLastError();
  if (*err != hipSuccess) return -1;
  if (sweeps_out) *sweeps_out = sweep + 1;
  return converged ? 0 : 1;
}

}  // namespace ef
