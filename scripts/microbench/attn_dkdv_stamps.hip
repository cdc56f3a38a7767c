// Per-wave phase timeline of k_attn_dkdv_seq (HSTU, hd 64) on bench-shaped
// ragged sequences, from 100 MHz s_memrealtime stamps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o build/attn_dkdv_stamps scripts/microbench/attn_dkdv_stamps.hip
//   build/attn_dkdv_stamps [B]
// Stamps per wave: 0 entry, 1 staging issued+written, 2 after the barrier,
// 3/4/5 after key tile 1/2/3, 6 exit.
#define GRK_DKDV_STAMPS 1
#include <algorithm>
#include <vector>

#include "../../tencent_recommendation_2025_amd/csrc/grk_attention_seq.hip"
#include "../../tencent_recommendation_2025_amd/csrc/grk_util.cpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 128, T = 201, H = 8, HD = 64, D = H * HD;
  const int N = B * T;
  bf16_t *pre, *dout, *dpre; uint8_t* kv; float* rab; int* rng; unsigned long long* drab;
  CK(hipMalloc(&pre, (size_t)N * 4 * D * 2)); CK(hipMalloc(&kv, N)); CK(hipMalloc(&rab, H * T * 4));
  CK(hipMalloc(&dout, (size_t)N * D * 2)); CK(hipMalloc(&dpre, (size_t)N * 4 * D * 2)); CK(hipMalloc(&rng, B * 12));
  CK(hipMemset(pre, 0x3c, (size_t)N * 4 * D * 2)); CK(hipMemset(dout, 0x3c, (size_t)N * D * 2)); CK(hipMemset(rab, 0, H * T * 4));
  std::vector<uint8_t> hv(N);
  std::vector<int> len(B);
  srand(1);
  for (int b = 0; b < B; ++b) { len[b] = 32 + rand() % (T - 31); for (int t = 0; t < T; ++t) hv[b * T + t] = t >= T - len[b]; }
  CK(hipMemcpy(kv, hv.data(), N, hipMemcpyHostToDevice));
  k_seq_ranges<<<(B + 3) / 4, 256>>>(kv, B, T, rng);
  k_seq_order<<<1, 1024>>>(B, T, rng);
  AttnParams p; memset(&p, 0, sizeof(p));
  p.kind = 1; p.B = B; p.H = H; p.T = T; p.precise = 1;
  p.q = pre + 2 * D; p.k = pre + 3 * D; p.v = pre + D; p.ldq = p.ldk = p.ldv = 4 * D;
  p.key_valid = kv; p.scale = 0.125f; p.inv_n = 1.0f / T; p.rab = rab; p.nb = T; p.act = 1; p.seq_range = rng;
  p.dout = dout; p.lddo = D; p.dk = dpre + 3 * D; p.dv = dpre + D; p.lddk = p.lddv = 4 * D; p.in_dt = 1;
  const int Tp = (T + 31) / 32 * 32;
  const size_t lds = SeqLds<64>::bytes(Tp);
  for (int it = 0; it < 3; ++it) launch_lds(k_attn_dkdv_seq<64, 1, 1>, dim3(B * H), 256, lds, 0, p);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  launch_lds(k_attn_dkdv_seq<64, 1, 1>, dim3(B * H), 256, lds, 0, p);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = B * H * 4;
  std::vector<unsigned long long> st((size_t)nw * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_dkdv_rt), st.size() * 8));
  std::vector<int> hr(B * 3);
  CK(hipMemcpy(hr.data(), rng, B * 12, hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int w = 0; w < nw; ++w) { t0 = std::min(t0, st[(size_t)w * 8]); t1 = std::max(t1, st[(size_t)w * 8 + 6]); }
  printf("B=%d: %.2f us kernel (events); stamps span %.2f us; LDS %zu B\n", B, ms * 1e3, (t1 - t0) / 100.0, lds);
  // per length class: averages (us) of staging, barrier wait, per tile, start offset, end
  const int edges[] = {32, 64, 96, 128, 160, 192, 202};
  for (int c = 0; c + 1 < 7; ++c) {
    double stg = 0, bar = 0, tile1 = 0, tot = 0, st0 = 0, end = 0; int n = 0, nt = 0;
    for (int w = 0; w < nw; ++w) {
      const int blk = w / 4, b = hr[3 * (blk / H) + 2];
      const int L = T - hr[3 * b];
      if (L < edges[c] || L >= edges[c + 1]) continue;
      unsigned long long* s = &st[(size_t)w * 8];
      stg += (s[1] - s[0]) / 100.0; bar += (s[2] - s[1]) / 100.0; tot += (s[6] - s[0]) / 100.0;
      st0 += (s[0] - t0) / 100.0; end += (s[6] - t0) / 100.0;
      if (s[3] > s[2] && s[3] - s[2] < 1000000) { tile1 += (s[3] - s[2]) / 100.0; ++nt; }
      ++n;
    }
    if (n) printf("  L in [%3d,%3d): %5d waves  start %6.2f  staging %5.2f  barrier %5.2f  tile1 %5.2f  wave total %6.2f  end %6.2f us\n",
                  edges[c], edges[c + 1], n, st0 / n, stg / n, bar / n, nt ? tile1 / nt : 0.0, tot / n, end / n);
  }
  return 0;
}
