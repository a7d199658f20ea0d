// Step timeline of conv_tk2 (ops.hip) on S3D base.3's (3,1,1) 192->192 conv
// at 8x28x28 (256 clips) from s_memtime stamps of every wave: after the
// previous step (0), after the wait + barrier (1), after the slice issue (2),
// after the step's MFMAs are issued (3).  GPU box:
//   hipcc --offload-arch=gfx950 -O3 -DTK2_STAMPS -I fac_fake_amd/csrc -I include \
//     -o tools/ubench/bin/tk2_ubench tools/ubench/tk2_ubench.hip && tools/ubench/bin/tk2_ubench
#include "../../fac_fake_amd/csrc/ops.hip"

#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  const int B = 256, D = 8, S = 784, Cin = argc > 1 ? atoi(argv[1]) : 192, Cout = Cin, KD = 3;
  const size_t nin = (size_t)B * D * S * Cin;
  std::vector<uint16_t> hin(nin);
  for (size_t i = 0; i < nin; ++i) hin[i] = 0x3c00 + (uint16_t)((i * 2654435761u >> 20) & 0x3ff);
  const int kp = KD * Cin;
  std::vector<uint16_t> hw((size_t)Cout * kp);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0x2000 + (uint16_t)((i * 40503u >> 6) & 0x3ff);
  uint16_t *din, *dw, *dout;
  float* db;
  (void)hipMalloc(&din, nin * 2);
  (void)hipMalloc(&dw, hw.size() * 2);
  (void)hipMalloc(&dout, nin * 2);
  (void)hipMalloc(&db, Cout * 4);
  (void)hipMemset(db, 0, Cout * 4);
  (void)hipMemcpy(din, hin.data(), nin * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  const int nunits = B * ((S + 15) / 16), nbk = Cout / 64, nslot = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    fac::conv_tk2<fac::BF16, 1, 3, 1, 2, 5><<<nslot * nbk, 512>>>(din, dw, db, dout, nunits, S, Cin, kp, Cout, 0, 1, nbk, nslot);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  printf("conv_tk2 (3,1,1) %d->%d, %d clips x 8 x %d: %.1f us\n", Cin, Cout, B, S, ms * 1e3);
  static unsigned long long st[4][64][8][4];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(fac::tk2_st), sizeof(st));
  for (int wg = 0; wg < 2; ++wg) {
    printf("wg %d, mean ticks over steps 8..55 per wave: [prev->barrier done] [issue] [reads+MFMA issue] [to next step]\n", wg);
    for (int w = 0; w < 8; ++w) {
      double a = 0, b = 0, c = 0, d = 0;
      int n = 0;
      for (int s = 8; s < 56; ++s, ++n) {
        a += (double)(st[wg][s][w][1] - st[wg][s][w][0]);
        b += (double)(st[wg][s][w][2] - st[wg][s][w][1]);
        c += (double)(st[wg][s][w][3] - st[wg][s][w][2]);
        d += (double)(st[wg][s + 1][w][0] - st[wg][s][w][3]);
      }
      printf("  w%d %6.0f %6.0f %6.0f %6.0f\n", w, a / n, b / n, c / n, d / n);
    }
  }
  return 0;
}
