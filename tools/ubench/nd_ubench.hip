// Step timeline of convnd_igemm (ops.hip) on ResVitKan (ResNet-50, 512 crops)
// layers from s_memtime stamps of every wave of the first 8 workgroups: at the
// step start (0), after the stage issue (1), after the step's fragment reads
// + MFMAs are issued (2), after the vmcnt/lgkmcnt wait (3); the barrier is
// (3) -> next (0).  GPU box:
//   hipcc --offload-arch=gfx950 -O3 -DND_STAMPS -I fac_fake_amd/csrc -I include \
//     -o tools/ubench/bin/nd_ubench tools/ubench/nd_ubench.hip && tools/ubench/bin/nd_ubench [layer]
#include "../../fac_fake_amd/csrc/ops.hip"

#include <cstdio>
#include <vector>

struct L {
  const char* name;
  int h, cin, cout, k, s, p;
};

int main(int argc, char** argv) {
  const L layers[] = {{"1x1/1 1024->512 @14", 14, 1024, 512, 1, 1, 0},
                      {"1x1/1 512->256 @28", 28, 512, 256, 1, 1, 0},
                      {"3x3/2 128->128 @56", 56, 128, 128, 3, 2, 1},
                      {"1x1/2 256->512 @56", 56, 256, 512, 1, 2, 0}};
  const int li = argc > 1 ? atoi(argv[1]) : 0;
  const L& l = layers[li];
  const int B = 512, ho = (l.h + 2 * l.p - l.k) / l.s + 1;
  const size_t nin = (size_t)B * l.h * l.h * l.cin, nout = (size_t)B * ho * ho * l.cout;
  int cp, kp;
  fac_conv_weight_layout(l.cout, l.cin, 1, l.k, l.k, &cp, &kp);
  std::vector<uint16_t> hin(nin), hw((size_t)cp * kp);
  for (size_t i = 0; i < nin; ++i) hin[i] = 0x3c00 + (uint16_t)((i * 2654435761u >> 20) & 0x3ff);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0x2000 + (uint16_t)((i * 40503u >> 6) & 0x3ff);
  uint16_t *din, *dw, *dout;
  float* db;
  (void)hipMalloc(&din, nin * 2);
  (void)hipMalloc(&dw, hw.size() * 2);
  (void)hipMalloc(&dout, nout * 2);
  (void)hipMalloc(&db, cp * 4);
  (void)hipMemset(db, 0, cp * 4);
  (void)hipMemcpy(din, hin.data(), nin * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  fac_conv_desc d{};
  d.dtype = FAC_DTYPE_BF16;
  d.in = din;
  d.n = B;
  d.d = 1;
  d.h = d.w = l.h;
  d.cin = l.cin;
  d.weight = dw;
  d.bias = db;
  d.cout = l.cout;
  d.k_pad = kp;
  d.kd = 1;
  d.kh = d.kw = l.k;
  d.sd = 1;
  d.sh = d.sw = l.s;
  d.pd = 0;
  d.ph = d.pw = l.p;
  d.od = 1;
  d.oh = d.ow = ho;
  d.out = dout;
  d.ldo = l.cout;
  d.flags = FAC_CONV_RELU;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    if (fac_conv_nd(&d, nullptr) != FAC_OK) {
      printf("fac_conv_nd failed\n");
      return 1;
    }
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  const int ksteps = kp / 64;
  printf("%s, %d crops: %.1f us, %d K steps\n", l.name, B, ms * 1e3, ksteps);
  static unsigned long long st[8][40][8][4];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(fac::nd_st), sizeof(st));
  const int s1 = 39;  // convnd_pt: stamps run over the workgroup's steps across tiles
  for (int wg = 0; wg < 3; ++wg) {
    printf("wg %d, mean ticks over steps 1..%d per wave: [0->1] [1->2] [2->3] [3->next 0]\n", wg, s1 - 1);
    for (int w = 0; w < 8; ++w) {
      double a = 0, b = 0, c = 0, e = 0;
      int n = 0;
      for (int s = 1; s < s1; ++s, ++n) {
        a += (double)(st[wg][s][w][1] - st[wg][s][w][0]);
        b += (double)(st[wg][s][w][2] - st[wg][s][w][1]);
        c += (double)(st[wg][s][w][3] - st[wg][s][w][2]);
        e += (double)(st[wg][s + 1][w][0] - st[wg][s][w][3]);
      }
      printf("  w%d %6.0f %6.0f %6.0f %6.0f   step0->1 start %llu\n", w, a / n, b / n, c / n, e / n,
             st[wg][1][w][0] - st[wg][0][w][0]);
    }
  }
  static unsigned long long ev[8][8][4];
  (void)hipMemcpyFromSymbol(ev, HIP_SYMBOL(fac::nd_ev), sizeof(ev));
  printf("per workgroup (wave 0 / max over waves): prologue, K loop, epilogue (ticks)\n");
  for (int wg = 0; wg < 8; ++wg) {
    unsigned long long a = 0, b = 0, c = 0;
    for (int w = 0; w < 8; ++w) {
      a = std::max(a, ev[wg][w][1] - ev[wg][w][0]);
      b = std::max(b, ev[wg][w][2] - ev[wg][w][1]);
      c = std::max(c, ev[wg][w][3] - ev[wg][w][2]);
    }
    printf("  wg %d  %6llu %6llu %6llu   max %6llu %6llu %6llu\n", wg, ev[wg][0][1] - ev[wg][0][0],
           ev[wg][0][2] - ev[wg][0][1], ev[wg][0][3] - ev[wg][0][2], a, b, c);
  }
  return 0;
}
