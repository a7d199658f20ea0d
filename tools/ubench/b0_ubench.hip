// Phase timeline of s3d_base0 (ops.hip, S3D's fused base.0) from s_memtime
// stamps (B0_STAMPS): per unit, mean ticks of each phase over workgroups 0-7,
// units 1-15, and the per-wave spread at the barriers.
// GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DB0_STAMPS -I fac_fake_amd/csrc -I include \
//     -o /tmp/b0_ubench tools/ubench/b0_ubench.hip && /tmp/b0_ubench
#include "../../fac_fake_amd/csrc/ops.hip"

#include <cstdio>
#include <vector>

int main() {
  const int n = 384, T = 16, H = 112, W = 112;
  std::vector<uint8_t> clip((size_t)n * 3 * T * H * W);
  for (size_t i = 0; i < clip.size(); ++i) clip[i] = (uint8_t)(i * 2654435761u >> 24);
  std::vector<uint16_t> ws(64 * 256), wt(64 * 448);
  for (size_t i = 0; i < ws.size(); ++i) ws[i] = 0x3c00 + (uint16_t)((i * 40503u >> 8) & 0x3f);
  for (size_t i = 0; i < wt.size(); ++i) wt[i] = 0x2c00 + (uint16_t)((i * 40503u >> 8) & 0x3f);
  std::vector<float> b(64, 0.01f);
  uint8_t* dclip;
  uint16_t *dws, *dwt, *dout;
  float *dbs, *dbt;
  (void)hipMalloc(&dclip, clip.size());
  (void)hipMalloc(&dws, ws.size() * 2);
  (void)hipMalloc(&dwt, wt.size() * 2);
  (void)hipMalloc(&dbs, 256);
  (void)hipMalloc(&dbt, 256);
  (void)hipMalloc(&dout, (size_t)n * 8 * 56 * 56 * 64 * 2);
  (void)hipMemcpy(dclip, clip.data(), clip.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dws, ws.data(), ws.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dwt, wt.data(), wt.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dbs, b.data(), 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dbt, b.data(), 256, hipMemcpyHostToDevice);
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int nunits = n * 196, grid = ncu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    fac::s3d_base0<fac::BF16><<<grid, 512, 0, 0>>>(dclip, dws, dbs, 256, dwt, dbt, 448, dout, nunits, H, W, 2, 1, 1);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  printf("s3d_base0 n=%d: %.1f us, %d units on %d workgroups (%.1f units each), %.0f ns per unit\n", n, ms * 1e3,
         nunits, grid, (double)nunits / grid, ms * 1e6 / ((double)nunits / grid));
  static unsigned long long st[8][16][8][8];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(fac::b0_st), sizeof(st));
  const char* nm[8] = {"start->A", "A:spatial", "->B", "B:S+cells", "->C", "C:temporal", "store", "->next"};
  double ph[8] = {0};
  int cnt = 0;
  for (int x = 0; x < 8; ++x)
    for (int k = 1; k < 15; ++k, ++cnt)
      for (int p = 0; p < 8; ++p)
        ph[p] += (double)((p < 7 ? st[x][k][0][p + 1] : st[x][k + 1][0][0]) - st[x][k][0][p]);
  printf("wave 0 mean ticks per unit:");
  double tot = 0;
  for (int p = 0; p < 8; ++p) {
    printf(" %s %.0f", nm[p], ph[p] / cnt);
    tot += ph[p] / cnt;
  }
  printf("  (sum %.0f)\n", tot);
  printf("per wave, barrier A -> spatial done / barrier C -> temporal done:");
  for (int w = 0; w < 8; ++w) {
    double a = 0, c = 0;
    for (int x = 0; x < 8; ++x)
      for (int k = 1; k < 15; ++k) {
        a += (double)(st[x][k][w][2] - st[x][k][0][1]);
        c += (double)(st[x][k][w][6] - st[x][k][0][5]);
      }
    printf(" w%d %.0f/%.0f", w, a / cnt, c / cnt);
  }
  printf("\n");
  return 0;
}
