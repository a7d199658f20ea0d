// Phase timeline of conv3x3_bn_relu's 112^2 tiles (conv.hip) from s_memtime
// stamps (CONV_STAMPS): per workgroup, wave 0..3, start / prologue landed /
// nine step barriers of chunk 0 / last chunk / staged / stored.
// GPU box:
//   hipcc --offload-arch=gfx950 -O3 -DCONV_STAMPS -I fac_fake_amd/csrc -I include \
//     -o /tmp/conv_ubench tools/ubench/conv_ubench.hip && /tmp/conv_ubench
#include "../../fac_fake_amd/csrc/conv.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

static void run(int H, int cin, int cout, bool pool, int B) {
  const size_t nin = (size_t)B * H * H * cin, nout = (size_t)B * H * H * cout;
  std::vector<uint16_t> hin(nin), hw((size_t)9 * cin * cout);
  for (size_t i = 0; i < nin; ++i) hin[i] = 0x3800 + (uint16_t)((i * 2654435761u >> 20) & 0x3ff);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0x2c00 + (uint16_t)((i * 40503u >> 8) & 0x3f);
  std::vector<float> bias(cout, 0.01f);
  uint16_t *din, *dw, *dout, *dz;
  float* db;
  (void)hipMalloc(&din, nin * 2);
  (void)hipMalloc(&dw, hw.size() * 2);
  (void)hipMalloc(&dout, nout * 2);
  (void)hipMalloc(&dz, 4096);
  (void)hipMalloc(&db, cout * 4);
  (void)hipMemset(dz, 0, 4096);
  (void)hipMemcpy(din, hin.data(), nin * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, bias.data(), cout * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  static unsigned long long st[16384][4][14];
  std::fill(&st[0][0][0], &st[0][0][0] + 16384 * 4 * 14, 0ull);
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(fac::conv_st), st, sizeof(st));
    (void)hipEventRecord(e0, 0);
    hipError_t err = fac::launch_conv3x3(1, din, dw, db, dout, B, H, H, cin, cout, pool, dz, 0, true, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (err != hipSuccess) { printf("launch failed %d\n", (int)err); return; }
  }
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(fac::conv_st), sizeof(st));
  int nbox = 0;
  while (nbox < 16384 && st[nbox][0][13]) ++nbox;
  unsigned long long t0 = ~0ull, t1 = 0;
  double ph[14] = {0}, life = 0;
  for (int x = 0; x < nbox; ++x) {
    t0 = std::min(t0, st[x][0][0]);
    t1 = std::max(t1, st[x][0][13]);
    for (int k = 1; k < 14; ++k) ph[k] += (double)(st[x][0][k] - st[x][0][k - 1]);
    life += (double)(st[x][0][13] - st[x][0][0]);
  }
  printf("conv %d^2 %d->%d%s B=%d: %.1f us, %d boxes, span %.0f ticks, mean box life %.0f ticks, boxes in flight %.1f/CU\n",
         H, cin, cout, pool ? " pool" : "", B, ms * 1e3, nbox, (double)(t1 - t0), life / nbox,
         life / (double)(t1 - t0) / 256.0);
  const char* nm[14] = {"", "prologue", "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "s8", "rest", "stage", "store"};
  printf("  wave 0 mean ticks:");
  for (int k = 1; k < 14; ++k) printf(" %s %.0f", nm[k], ph[k] / nbox);
  printf("\n  step 0..8 per wave (mean, barrier to barrier):");
  for (int w = 0; w < 4; ++w) {
    double sm = 0;
    for (int x = 0; x < nbox; ++x) sm += (double)(st[x][w][10] - st[x][w][1]);
    printf(" w%d %.0f", w, sm / nbox / 9);
  }
  // dispatch ramp: starts in the first / last 10 % of boxes
  std::vector<double> starts(nbox);
  for (int x = 0; x < nbox; ++x) starts[x] = (double)(st[x][0][0] - t0);
  std::sort(starts.begin(), starts.end());
  printf("\n  start ticks: p10 %.0f p50 %.0f p90 %.0f\n", starts[nbox / 10], starts[nbox / 2], starts[nbox * 9 / 10]);
  (void)hipFree(din);
  (void)hipFree(dw);
  (void)hipFree(dout);
  (void)hipFree(dz);
  (void)hipFree(db);
}

int main() {
  run(112, 32, 64, false, 256);
  run(112, 64, 64, false, 256);
  run(112, 64, 64, true, 256);
  run(56, 64, 128, false, 256);
  run(14, 512, 512, false, 256);
  return 0;
}
