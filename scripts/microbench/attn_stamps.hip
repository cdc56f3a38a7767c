// Per-phase cycle breakdown of k_attn_fwd_seq (HSTU) via s_memtime stamps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o build/attn_stamps scripts/microbench/attn_stamps.hip
//   build/attn_stamps [B]
// Stamps per wave: 0 entry, 1 after seq_info, 2 staging issued+written,
// 3 after the barrier, 4/5 after tile 1/2, 6 exit.
#define GRK_ATTN_STAMPS 1
#include <vector>

#include "../../tencent_recommendation_2025_amd/csrc/grk_attention_seq.hip"
#include "../../tencent_recommendation_2025_amd/csrc/grk_util.cpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, T = 201, H = 8, HD = 64, D = H * HD;
  const int N = B * T;
  bf16_t* pre; uint8_t* kv; float* rab; bf16_t* out; int* rng;
  CK(hipMalloc(&pre, (size_t)N * 4 * D * 2)); CK(hipMalloc(&kv, N)); CK(hipMalloc(&rab, H * T * 4));
  CK(hipMalloc(&out, (size_t)N * D * 2)); CK(hipMalloc(&rng, B * 8));
  CK(hipMemset(pre, 0x3c, (size_t)N * 4 * D * 2)); CK(hipMemset(rab, 0, H * T * 4));
  std::vector<uint8_t> hv(N);
  srand(1);
  for (int b = 0; b < B; ++b) { int len = 32 + rand() % (T - 31); for (int t = 0; t < T; ++t) hv[b * T + t] = t >= T - len; }
  CK(hipMemcpy(kv, hv.data(), N, hipMemcpyHostToDevice));
  k_seq_ranges<<<(B + 3) / 4, 256>>>(kv, B, T, rng);
  AttnParams p; memset(&p, 0, sizeof(p));
  p.kind = 1; p.B = B; p.H = H; p.T = T;
  p.q = pre + 2 * D; p.k = pre + 3 * D; p.v = pre + D; p.ldq = p.ldk = p.ldv = 4 * D;
  p.key_valid = kv; p.scale = 0.125f; p.inv_n = 1.0f / T; p.rab = rab; p.nb = T; p.act = 1; p.seq_range = rng;
  p.out = out; p.ldo = D;
  const int Tp = (T + 31) / 32 * 32;
  const size_t lds = SeqLds<64>::bytes(Tp);
  for (int it = 0; it < 3; ++it) k_attn_fwd_seq<64, 1, 0><<<B * H, 256, lds>>>(p);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  k_attn_fwd_seq<64, 1, 0><<<B * H, 256, lds>>>(p);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = B * H * 4;
  std::vector<unsigned long long> st((size_t)nw * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_attn_stamps), st.size() * 8));
  double acc[8] = {0}; int cnt[8] = {0};
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int w = 0; w < nw; ++w) {
    unsigned long long* s = &st[(size_t)w * 8];
    t0 = std::min(t0, s[0]); t1 = std::max(t1, s[6]);
    const int order[] = {0, 1, 2, 3, 4, 5, 6};
    for (int k = 1; k < 7; ++k) {
      int prev = k - 1;
      if (k == 6 && s[5] < s[4]) prev = 4;  // wave with one tile: no stamp 5 this launch
      if (k == 5 && s[5] < s[4]) continue;
      if (s[k] >= s[prev]) { acc[k] += (double)(s[k] - s[prev]); cnt[k]++; }
    }
    (void)order;
  }
  const char* names[] = {"", "seq_info", "staging (issue+wait+write)", "barrier", "tile A", "tile B", "exit"};
  printf("B=%d: %.1f us kernel; stamp span %.0f ticks\n", B, ms * 1e3, (double)(t1 - t0));
  for (int k = 1; k < 7; ++k) printf("  %-28s %9.0f ticks avg over %d waves\n", names[k], cnt[k] ? acc[k] / cnt[k] : 0, cnt[k]);
  return 0;
}
