// Microbenchmark (diagnostic, not product): L2 write requests and time of the
// store shapes the fast step can use for its 64-B state/message records,
// written through a scattered list as the work lists do.  Run under
// rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum to count requests per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

struct alignas(16) Rec { uint4 c[4]; };

// P1: one lane per record, 4 x 16-B stores (the current fast step)
__global__ void p1_lane_record(Rec* out, const unsigned* perm, unsigned n) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Rec* r = out + perm[i];
  for (int c = 0; c < 4; c++) r->c[c] = make_uint4(i, c, 1, 2);
}
// P2: four lanes per record, one 16-B chunk each (wave-cooperative)
__global__ void p2_quad_record(Rec* out, const unsigned* perm, unsigned n) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * n) return;
  Rec* r = out + perm[i >> 2];
  r->c[i & 3] = make_uint4(i, 7, 1, 2);
}
// P3: one lane per record, one 16-B store (a dirty chunk only)
__global__ void p3_lane_chunk(Rec* out, const unsigned* perm, unsigned n) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[perm[i]].c[0] = make_uint4(i, 3, 1, 2);
}
// P4: sub-wave of 3 lanes per group, each lane its own (adjacent) record, 4 stores
__global__ void p4_group_lane_record(Rec* out, const unsigned* gperm, unsigned ngroups) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned w = threadIdx.x & 63;
  if (w >= 63) return;
  unsigned g = (blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) / 64 * 21 + w / 3;
  if (g >= ngroups) return;
  Rec* r = out + (size_t)gperm[g] * 3 + (w % 3);
  for (int c = 0; c < 4; c++) r->c[c] = make_uint4(i, c, 1, 2);
}
// P5: sub-wave of 12 lanes per group writes the group's 3 adjacent records,
// 16 B per lane, one instruction (transposed)
__global__ void p5_group_transposed(Rec* out, const unsigned* gperm, unsigned ngroups) {
  unsigned w = threadIdx.x & 63;
  if (w >= 60) return;
  unsigned g = (blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) / 64 * 5 + w / 12;
  if (g >= ngroups) return;
  uint4* base = (uint4*)(out + (size_t)gperm[g] * 3);
  base[w % 12] = make_uint4(w, 9, 1, 2);
}
// P6: one lane per record, 2 x 16-B stores (a 32-B compact record)
__global__ void p6_lane_half(Rec* out, const unsigned* perm, unsigned n) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Rec* r = out + perm[i];
  r->c[0] = make_uint4(i, 0, 1, 2);
  r->c[1] = make_uint4(i, 1, 1, 2);
}

int main() {
  const unsigned NREC = 3u << 20;       // 3M records (C4 replicas), 192 MB
  const unsigned NW = 300000;           // active replica-steps per round
  const unsigned NG = NW / 3;           // active groups
  std::vector<unsigned> perm(NREC / 3), rperm(NW);
  std::mt19937 rng(1);
  for (unsigned i = 0; i < perm.size(); i++) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<unsigned> gsorted(perm.begin(), perm.begin() + NG);
  std::sort(gsorted.begin(), gsorted.end());  // work lists come out in replica order
  for (unsigned i = 0; i < NW; i++) rperm[i] = gsorted[i / 3] * 3 + i % 3;
  Rec* out;
  unsigned *d_rperm, *d_gperm;
  hipMalloc(&out, sizeof(Rec) * (size_t)NREC);
  hipMalloc(&d_rperm, NW * 4);
  hipMalloc(&d_gperm, NG * 4);
  hipMemcpy(d_rperm, rperm.data(), NW * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_gperm, gsorted.data(), NG * 4, hipMemcpyHostToDevice);
  hipMemset(out, 0, sizeof(Rec) * (size_t)NREC);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto t = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; w++) launch();
    hipEventRecord(a);
    for (int w = 0; w < 20; w++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-24s %8.2f us/launch\n", name, ms * 1000 / 20);
  };
  const unsigned B = 256;
  t("p1_lane_record", [&] { p1_lane_record<<<(NW + B - 1) / B, B>>>(out, d_rperm, NW); });
  t("p2_quad_record", [&] { p2_quad_record<<<(4 * NW + B - 1) / B, B>>>(out, d_rperm, NW); });
  t("p3_lane_chunk", [&] { p3_lane_chunk<<<(NW + B - 1) / B, B>>>(out, d_rperm, NW); });
  t("p6_lane_half", [&] { p6_lane_half<<<(NW + B - 1) / B, B>>>(out, d_rperm, NW); });
  t("p4_group_lane_record", [&] {
    p4_group_lane_record<<<((NG + 20) / 21 * 64 + B - 1) / B, B>>>(out, d_gperm, NG);
  });
  t("p5_group_transposed", [&] {
    p5_group_transposed<<<((NG + 4) / 5 * 64 + B - 1) / B, B>>>(out, d_gperm, NG);
  });
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
