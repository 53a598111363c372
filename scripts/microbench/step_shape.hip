// Microbenchmark (diagnostic, not product): the memory shape of one C4 fast
// step per lane — scattered loads of Hot/Core/count row/two inbound messages,
// a little arithmetic, scattered stores of Hot/Upd chunk/Core chunk/count row
// and two outbound 64-B messages — with the message stores done
//   A: one lane per message, four 16-B stores (the fast step today),
//   B: through LDS, four lanes per message, one 16-B chunk each,
// at 2 and 4 resident waves per SIMD (LDS padding caps the blocks per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

struct alignas(16) Msg { uint4 c[4]; };
struct alignas(16) Hot { uint4 c[2]; };
struct alignas(16) Core { uint4 c[4]; };

template <bool COOP>
__global__ __launch_bounds__(256) void k_shape(Hot* hot, Core* core, uint4* upd, uint4* cnt,
                                               Msg* msgs_in, Msg* msgs_out, const unsigned* list,
                                               unsigned n, unsigned maxm) {
  extern __shared__ uint4 pad_lds[];
  __shared__ uint4 stage[4][2][64][4];   // [wave][message j][lane][chunk]
  __shared__ unsigned long long sdst[4][2][64];
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  const unsigned r = act ? list[i] : 0;
  const unsigned g = r / 3, k = r % 3;
  // gather
  Hot h = hot[r];
  Core c = core[r];
  uint4 cw = cnt[g * 3 + (k + 1) % 3];
  Msg a = msgs_in[((size_t)(g * 3 + (k + 1) % 3) * 3 + k) * maxm];
  Msg b = msgs_in[((size_t)(g * 3 + (k + 2) % 3) * 3 + k) * maxm];
  // compute
  uint4 x = h.c[0];
  x.x += c.c[0].x + cw.x + a.c[1].y + b.c[2].z;
  x.y ^= c.c[1].y + a.c[0].x;
  h.c[0] = x;
  c.c[1].x += a.c[3].w + b.c[0].x;
  Msg o0 = a, o1 = b;
  o0.c[0].x ^= x.x;
  o1.c[0].x ^= x.y;
  if (act) {
    hot[r] = h;
    upd[r * 4 + 3] = x;
    core[r].c[1] = c.c[1];
    cnt[r] = cw;
  }
  const size_t d0 = ((size_t)(g * 3 + k) * 3 + (k + 1) % 3) * maxm + (maxm > 1);
  const size_t d1 = ((size_t)(g * 3 + k) * 3 + (k + 2) % 3) * maxm + (maxm > 1);
  if (!COOP) {
    if (act) {
      msgs_out[d0] = o0;
      msgs_out[d1] = o1;
    }
  } else {
    for (int q = 0; q < 4; q++) {
      stage[w][0][lane][q] = o0.c[q];
      stage[w][1][lane][q] = o1.c[q];
    }
    sdst[w][0][lane] = act ? d0 : ~0ull;
    sdst[w][1][lane] = act ? d1 : ~0ull;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < 2; j++) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const unsigned src = q * 16 + lane / 4, ch = lane & 3;
        const unsigned long long dst = sdst[w][j][src];
        if (dst != ~0ull) msgs_out[dst].c[ch] = stage[w][j][src][ch];
      }
    }
  }
  if (act && pad_lds[0].x == 12345u) hot[0].c[1].x = 1;  // keep the padding alive
}

int main() {
  const unsigned G = 1u << 20, R = 3 * G, NW = 300000, NG = NW / 3, MAXM = 12;
  std::vector<unsigned> perm(G), list(NW);
  std::mt19937 rng(1);
  for (unsigned i = 0; i < G; i++) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<unsigned> gs(perm.begin(), perm.begin() + NG);
  std::sort(gs.begin(), gs.end());
  // leaders first, then followers, as the work lists are laid out
  for (unsigned i = 0; i < NG; i++) list[i] = gs[i] * 3;
  for (unsigned i = 0; i < NG; i++) { list[NG + 2 * i] = gs[i] * 3 + 1; list[NG + 2 * i + 1] = gs[i] * 3 + 2; }
  Hot* hot; Core* core; uint4 *upd, *cnt; Msg *mi, *mo; unsigned* dl;
  hipMalloc(&hot, sizeof(Hot) * (size_t)R);
  hipMalloc(&core, sizeof(Core) * (size_t)R);
  hipMalloc(&upd, 64 * (size_t)R);
  hipMalloc(&cnt, 16 * (size_t)R);
  hipMalloc(&mi, sizeof(Msg) * (size_t)G * 9 * MAXM);
  hipMalloc(&mo, sizeof(Msg) * (size_t)G * 9 * MAXM);
  hipMalloc(&dl, NW * 4);
  hipMemcpy(dl, list.data(), NW * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned B = 256, grid = (NW + B - 1) / B;
  auto t = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; w++) launch();
    hipEventRecord(e0);
    for (int w = 0; w < 20; w++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.2f us/launch\n", name, ms * 1000 / 20);
  };
  // dynamic LDS padding: ~70 KB per block -> 2 blocks (8 waves) per CU; 30 KB -> 4 blocks
  // message footprint: the (sender, destination) list capacity sets how far
  // apart the lists are (the C4 engine uses 12 slots of 64 B)
  for (unsigned mm : {12u, 4u, 1u}) {
    char nm[64];
    snprintf(nm, sizeof(nm), "A direct maxm %u", mm);
    t(nm, [&] { hipLaunchKernelGGL(k_shape<false>, dim3(grid), dim3(B), 0, 0, hot, core, upd, cnt, mi, mo, dl, NW, mm); });
    snprintf(nm, sizeof(nm), "B coop   maxm %u", mm);
    t(nm, [&] { hipLaunchKernelGGL(k_shape<true>, dim3(grid), dim3(B), 0, 0, hot, core, upd, cnt, mi, mo, dl, NW, mm); });
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
