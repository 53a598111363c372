// Microbenchmark (diagnostic, not product): which part of the fast step's
// memory shape (scripts/microbench/step_shape.hip) costs what.  One lane per
// replica of a sorted C4-like work list (300k replica-steps over 1M groups):
//   L  : the gather only (Hot 32 B, Core 64 B, count row 16 B, 2 messages),
//   LQ : the same gather with 4 lanes per 64-B record (Core, messages) and
//        2 per Hot row, each lane one 16-B chunk, exchanged through LDS,
//   S  : the scatter only (Hot, Upd chunk, Core chunk, count row, 2 messages),
//   SQ : the scatter with every record written by 1/2/4 cooperating lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

struct alignas(16) Msg { uint4 c[4]; };

__device__ __forceinline__ void sink(uint4 v, uint4* out) {
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) out[0] = v;
}

// L: per-lane gather
__global__ __launch_bounds__(256) void k_L(const uint4* hot, const uint4* core, const uint4* cnt,
                                           const Msg* mi, const unsigned* list, unsigned n,
                                           unsigned maxm, uint4* out) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned r = list[i], g = r / 3, k = r % 3;
  uint4 a = hot[r * 2], b = hot[r * 2 + 1];
  uint4 c0 = core[r * 4], c1 = core[r * 4 + 1], c2 = core[r * 4 + 2], c3 = core[r * 4 + 3];
  uint4 w = cnt[g * 3 + (k + 1) % 3];
  const Msg m0 = mi[((size_t)(g * 3 + (k + 1) % 3) * 3 + k) * maxm];
  const Msg m1 = mi[((size_t)(g * 3 + (k + 2) % 3) * 3 + k) * maxm];
  uint4 x;
  x.x = a.x + b.y + c0.x + c1.y + c2.z + c3.w + w.x + m0.c[0].x + m0.c[1].y + m0.c[2].z + m0.c[3].w;
  x.y = m1.c[0].x + m1.c[1].y + m1.c[2].z + m1.c[3].w;
  x.z = x.w = 0;
  sink(x, out);
}

// LQ: cooperative gather: row j of the wave is loaded by lanes 4j..4j+3 (16 B
// each), 16 rows per instruction; results land in LDS rows
__global__ __launch_bounds__(256) void k_LQ(const uint4* hot, const uint4* core, const uint4* cnt,
                                            const Msg* mi, const unsigned* list, unsigned n,
                                            unsigned maxm, uint4* out) {
  __shared__ uint4 s[4][64][13];  // per lane: hot 2, core 4, 2 msgs 8 (w loaded directly)
  const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  const unsigned r = act ? list[i] : 0, g = r / 3, k = r % 3;
  const size_t a0 = ((size_t)(g * 3 + (k + 1) % 3) * 3 + k) * maxm;
  const size_t a1 = ((size_t)(g * 3 + (k + 2) % 3) * 3 + k) * maxm;
  const unsigned long long act_m = __ballot(act);
  // core: 4 instructions, each covering 16 rows
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const unsigned j = q * 16 + lane / 4, ch = lane & 3;
    const unsigned rj = __shfl(r, j, 64);
    if ((act_m >> j) & 1) s[wv][j][2 + ch] = core[rj * 4 + ch];
  }
  // hot: 2 instructions of 32 rows
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const unsigned j = q * 32 + lane / 2, ch = lane & 1;
    const unsigned rj = __shfl(r, j, 64);
    if ((act_m >> j) & 1) s[wv][j][ch] = hot[rj * 2 + ch];
  }
#pragma unroll
  for (int mm = 0; mm < 2; mm++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const unsigned j = q * 16 + lane / 4, ch = lane & 3;
      const unsigned long long aj = __shfl((unsigned long long)(mm ? a1 : a0), j, 64);
      if ((act_m >> j) & 1) s[wv][j][6 + mm * 4 + ch] = mi[aj].c[ch];
    }
  }
  uint4 w = cnt[g * 3 + (k + 1) % 3];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (!act) return;
  uint4 x;
  x.x = s[wv][lane][0].x + s[wv][lane][1].y + s[wv][lane][2].x + s[wv][lane][5].w + w.x +
        s[wv][lane][6].x + s[wv][lane][9].w;
  x.y = s[wv][lane][10].x + s[wv][lane][13 - 1].w;
  x.z = x.w = 0;
  sink(x, out);
}

// S: per-lane scatter
__global__ __launch_bounds__(256) void k_S(uint4* hot, uint4* core, uint4* upd, uint4* cnt,
                                           Msg* mo, const unsigned* list, unsigned n,
                                           unsigned maxm) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned r = list[i], g = r / 3, k = r % 3;
  const uint4 v = make_uint4(i, r, g, k);
  hot[r * 2] = v;
  hot[r * 2 + 1] = v;
  upd[r * 4 + 3] = v;
  core[r * 4 + 1] = v;
  cnt[r] = v;
  Msg m;
  for (int q = 0; q < 4; q++) m.c[q] = v;
  mo[((size_t)(g * 3 + k) * 3 + (k + 1) % 3) * maxm + 1] = m;
  mo[((size_t)(g * 3 + k) * 3 + (k + 2) % 3) * maxm + 1] = m;
}

// SQ: cooperative scatter (Hot rows by lane pairs, messages by lane quads; the
// single 16-B chunks stay one lane each)
__global__ __launch_bounds__(256) void k_SQ(uint4* hot, uint4* core, uint4* upd, uint4* cnt,
                                            Msg* mo, const unsigned* list, unsigned n,
                                            unsigned maxm) {
  const unsigned lane = threadIdx.x & 63;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  const unsigned r = act ? list[i] : 0, g = r / 3, k = r % 3;
  const unsigned long long am = __ballot(act);
  const uint4 v = make_uint4(i, r, g, k);
  if (act) {
    upd[r * 4 + 3] = v;
    core[r * 4 + 1] = v;
    cnt[r] = v;
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const unsigned j = q * 32 + lane / 2, ch = lane & 1;
    const unsigned rj = __shfl(r, j, 64);
    if ((am >> j) & 1) hot[rj * 2 + ch] = v;
  }
  const size_t d0 = ((size_t)(g * 3 + k) * 3 + (k + 1) % 3) * maxm + 1;
  const size_t d1 = ((size_t)(g * 3 + k) * 3 + (k + 2) % 3) * maxm + 1;
#pragma unroll
  for (int mm = 0; mm < 2; mm++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const unsigned j = q * 16 + lane / 4, ch = lane & 3;
      const unsigned long long dj = __shfl((unsigned long long)(mm ? d1 : d0), j, 64);
      if ((am >> j) & 1) mo[dj].c[ch] = v;
    }
  }
}

// LS: gather then scatter in one lane (the step's shape); `dis` = the scatter
// goes to a second copy of the planes instead of the rows just read
__global__ __launch_bounds__(256) void k_LS(const uint4* hot, const uint4* core, const uint4* cnt,
                                            const Msg* mi, uint4* whot, uint4* wcore, uint4* upd,
                                            uint4* wcnt, Msg* mo, const unsigned* list, unsigned n,
                                            unsigned maxm) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned r = list[i], g = r / 3, k = r % 3;
  uint4 a = hot[r * 2], b = hot[r * 2 + 1];
  uint4 c0 = core[r * 4], c1 = core[r * 4 + 1], c2 = core[r * 4 + 2], c3 = core[r * 4 + 3];
  uint4 w = cnt[g * 3 + (k + 1) % 3];
  const Msg m0 = mi[((size_t)(g * 3 + (k + 1) % 3) * 3 + k) * maxm];
  const Msg m1 = mi[((size_t)(g * 3 + (k + 2) % 3) * 3 + k) * maxm];
  uint4 v;
  v.x = a.x + b.y + c0.x + c1.y + c2.z + c3.w + w.x + m0.c[0].x + m0.c[1].y + m0.c[2].z + m0.c[3].w;
  v.y = m1.c[0].x + m1.c[1].y + m1.c[2].z + m1.c[3].w;
  v.z = i;
  v.w = r;
  whot[r * 2] = v;
  whot[r * 2 + 1] = v;
  upd[r * 4 + 3] = v;
  wcore[r * 4 + 1] = v;
  wcnt[r] = v;
  Msg m;
  for (int q = 0; q < 4; q++) m.c[q] = v;
  mo[((size_t)(g * 3 + k) * 3 + (k + 1) % 3) * maxm + 1] = m;
  mo[((size_t)(g * 3 + k) * 3 + (k + 2) % 3) * maxm + 1] = m;
}

int main() {
  const unsigned G = 1u << 20, R = 3 * G, NW = 300000, NG = NW / 3, MAXM = 12;
  std::vector<unsigned> perm(G), list(NW);
  std::mt19937 rng(1);
  for (unsigned i = 0; i < G; i++) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<unsigned> gs(perm.begin(), perm.begin() + NG);
  std::sort(gs.begin(), gs.end());
  for (unsigned i = 0; i < NG; i++) list[i] = gs[i] * 3;
  for (unsigned i = 0; i < NG; i++) { list[NG + 2 * i] = gs[i] * 3 + 1; list[NG + 2 * i + 1] = gs[i] * 3 + 2; }
  uint4 *hot, *core, *upd, *cnt, *out; Msg *mi, *mo; unsigned* dl;
  (void)hipMalloc(&hot, 32 * (size_t)R);
  (void)hipMalloc(&core, 64 * (size_t)R);
  (void)hipMalloc(&upd, 64 * (size_t)R);
  (void)hipMalloc(&cnt, 16 * (size_t)R);
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&mi, sizeof(Msg) * (size_t)G * 9 * MAXM);
  (void)hipMalloc(&mo, sizeof(Msg) * (size_t)G * 9 * MAXM);
  (void)hipMalloc(&dl, NW * 4);
  (void)hipMemcpy(dl, list.data(), NW * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const unsigned B = 256, grid = (NW + B - 1) / B;
  auto t = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; w++) launch();
    (void)hipEventRecord(e0);
    for (int w = 0; w < 20; w++) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-8s %8.2f us/launch\n", name, ms * 1000 / 20);
  };
  t("L", [&] { hipLaunchKernelGGL(k_L, dim3(grid), dim3(B), 0, 0, hot, core, cnt, mi, dl, NW, MAXM, out); });
  t("LQ", [&] { hipLaunchKernelGGL(k_LQ, dim3(grid), dim3(B), 0, 0, hot, core, cnt, mi, dl, NW, MAXM, out); });
  t("S", [&] { hipLaunchKernelGGL(k_S, dim3(grid), dim3(B), 0, 0, hot, core, upd, cnt, mo, dl, NW, MAXM); });
  t("SQ", [&] { hipLaunchKernelGGL(k_SQ, dim3(grid), dim3(B), 0, 0, hot, core, upd, cnt, mo, dl, NW, MAXM); });
  uint4 *hot2, *core2, *cnt2;
  (void)hipMalloc(&hot2, 32 * (size_t)R);
  (void)hipMalloc(&core2, 64 * (size_t)R);
  (void)hipMalloc(&cnt2, 16 * (size_t)R);
  t("LS same", [&] { hipLaunchKernelGGL(k_LS, dim3(grid), dim3(B), 0, 0, hot, core, cnt, mi, hot, core, upd, cnt, mo, dl, NW, MAXM); });
  t("LS disj", [&] { hipLaunchKernelGGL(k_LS, dim3(grid), dim3(B), 0, 0, hot, core, cnt, mi, hot2, core2, upd, cnt2, mo, dl, NW, MAXM); });
  t("L+S", [&] {
    hipLaunchKernelGGL(k_L, dim3(grid), dim3(B), 0, 0, hot, core, cnt, mi, dl, NW, MAXM, out);
    hipLaunchKernelGGL(k_S, dim3(grid), dim3(B), 0, 0, hot, core, upd, cnt, mo, dl, NW, MAXM);
  });
  (void)hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
