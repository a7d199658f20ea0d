// Phase timeline of the fused stem kernel (stem224.hip) from s_memtime
// stamps taken by wave 0 right after each of the five per-box barriers.
// GPU box:
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-atomic-optimizer-strategy=None -DSTEM_STAMPS -I fac_fake_amd/csrc -I include \
//     -o /tmp/stem_ubench tools/ubench/stem_ubench.hip && /tmp/stem_ubench
#include "../../fac_fake_amd/csrc/stem224.hip"

#include <cstdio>
#include <vector>

int main() {
  const int B = 256;
  std::vector<uint8_t> hin((size_t)B * 224 * 224 * 3);
  for (size_t i = 0; i < hin.size(); ++i) hin[i] = (uint8_t)(i * 2654435761u >> 24);
  std::vector<uint16_t> w1(32 * 64), w2(9 * 32 * 32), w3(9 * 32 * 32);
  for (size_t i = 0; i < w1.size(); ++i) w1[i] = 0x3c00 + (i * 40503u >> 8) % 64;
  for (size_t i = 0; i < w2.size(); ++i) w2[i] = w3[i] = 0x2c00 + (i * 40503u >> 8) % 64;
  std::vector<float> bias(32, 0.01f);
  uint8_t* din;
  uint16_t *dw1, *dw2, *dw3, *dout;
  float* db;
  (void)hipMalloc(&din, hin.size());
  (void)hipMalloc(&dw1, w1.size() * 2);
  (void)hipMalloc(&dw2, w2.size() * 2);
  (void)hipMalloc(&dw3, w3.size() * 2);
  (void)hipMalloc(&db, 128);
  (void)hipMalloc(&dout, (size_t)B * 112 * 112 * 32 * 2);
  (void)hipMemcpy(din, hin.data(), hin.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dw1, w1.data(), w1.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dw2, w2.data(), w2.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dw3, w3.data(), w3.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, bias.data(), 128, hipMemcpyHostToDevice);
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    (void)fac::launch_stem224(1, true, din, dw1, db, dw2, db, dw3, db, dout, B, ncu, 0, nullptr);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  printf("stem224 B=%d: %.1f us\n", B, ms * 1e3);
  static unsigned long long st[4][32][8][8];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(fac::stem_st), sizeof(st));
  const char* nm[5] = {"A stage", "B conv1", "C conv2", "D conv3", "out"};
  for (int wg = 0; wg < 2; ++wg) {
    printf("wg %d: mean s_memtime ticks per box, phase = barrier to barrier (wave 0):", wg);
    double sum[5] = {0};
    int n = 0;
    for (int j = 1; j < 31; ++j, ++n)
      for (int k = 0; k < 5; ++k) sum[k] += (double)((k < 4 ? st[wg][j][0][k + 1] : st[wg][j + 1][0][0]) - st[wg][j][0][k]);
    for (int k = 0; k < 5; ++k) printf("  %s %.0f", nm[k], sum[k] / n);
    printf("\n  per wave, barrier -> end of conv1 MFMAs:");
    for (int w = 0; w < 8; ++w) {
      double t1 = 0;
      for (int j = 1; j < 31; ++j) t1 += (double)(st[wg][j][w][7] - st[wg][j][0][1]);
      printf("  w%d %.0f", w, t1 / n);
    }
    printf("\n  per wave, barrier -> end of taps: conv2 / conv3:");
    for (int w = 0; w < 8; ++w) {
      double t2 = 0, t3 = 0;
      for (int j = 1; j < 31; ++j) {
        t2 += (double)(st[wg][j][w][5] - st[wg][j][0][2]);
        t3 += (double)(st[wg][j][w][6] - st[wg][j][0][3]);
      }
      printf("  w%d %.0f/%.0f", w, t2 / n, t3 / n);
    }
    printf("\n");
  }
  return 0;
}
