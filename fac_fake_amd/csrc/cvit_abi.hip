// C ABI (include/fac_cvit.h) and host orchestration of the CViT forward.
//
// Weight handling mirrors what the reference does implicitly at every call:
// eval-mode BatchNorm2d (cvit.py:89..146) is folded into the preceding conv
// once at load time (s = gamma / sqrt(var + eps); W' = W*s; b' = (b-mean)*s +
// beta), conv weights are repacked into per-(n-block, 32-channel chunk, tap)
// [BN][32] slices for the conv kernel, and linear weights are converted to
// the 16-bit operand type.  LayerNorm params, the CLS/pos embeddings and the
// final 2048->2 layer stay fp32.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/fac_cvit.h"
#include "common.hpp"

namespace fac {
void set_conv_ring9(int v);
int conv_block_n(int H, int cout);
void set_nd_pt_wide(int v);
void set_gemm_small(int max_m, int variant);
void set_nd_occ3(int v);
void set_pool_roll(int v);
void set_pool_win(int v);
void set_pool3_zg(int v);
void set_pool_lds14(int v);
void set_pw_res(int v);
void set_tk_wreg(int v);
void set_pool3_g(int v);
void pack_conv3x3(int dtype, int H, int ci, int co, const float* w, uint16_t* out, int bn = 0);
void pack_stem_conv1(int dtype, const float* w, uint16_t* out);
hipError_t launch_conv3x3(int dtype, const uint16_t* in, const uint16_t* wpk, const float* bias, uint16_t* out,
                          int B, int H, int W, int Cin, int Cout, bool pool, const uint16_t* zero16, hipStream_t st, bool relu = true,
                          int bn = 0);
hipError_t launch_conv1(int dtype, bool u8, const void* in, const uint16_t* w1, const float* bias, uint16_t* out,
                        int B, int H, int W, hipStream_t st);
hipError_t launch_gemm(int dtype, int epi, const uint16_t* A, int lda, const uint16_t* W, int ldw, const float* bias,
                       void* out, int ldo, int M, int N, int K, int splits, hipStream_t st, int variant = -1);
hipError_t launch_embed_finalize_ln(int dtype, const float* slab, int S, int B, const float* bias, const float* cls,
                                    const float* pos, const int32_t* pidx, float* x, const float* g, const float* bt,
                                    uint16_t* y, int* err, int seq, hipStream_t st);
hipError_t launch_layernorm(int dtype, const float* x, const float* g, const float* b, uint16_t* y, int R,
                            hipStream_t st);
hipError_t launch_gather_cls(int dtype, const float* x, uint16_t* c, int B, hipStream_t st);
hipError_t launch_resid_layernorm(int dtype, float* x, const float* slab, int S, const float* bias, const float* g,
                                 const float* b, uint16_t* y, int R, hipStream_t st, float eps = 1e-5f);
hipError_t launch_resid_cls(int dtype, const float* x, const float* slab, int S, const float* bias, uint16_t* c, int B,
                            hipStream_t st);
hipError_t launch_attention2(int dtype, const float* qkv, uint16_t* o, int B, float scale, hipStream_t st);
hipError_t launch_head_out(const float* hid, const float* w2, const float* b2, float* logits, float* probs, int B,
                           hipStream_t st);
hipError_t launch_video_score(const float* logits, int n, float* score, hipStream_t st);
hipError_t launch_video_score_seg(const float* logits, const int* seg, int nv, float* score, hipStream_t st);
hipError_t launch_crop_resize(const uint8_t* frames, int n_frames, int H, int W, const int32_t* boxes, int n_boxes,
                              uint8_t* crops, hipStream_t st);
hipError_t launch_stem224(int dtype, bool u8, const void* in, const uint16_t* w1, const float* b1, const uint16_t* w2,
                          const float* b2, const uint16_t* w3, const float* b3, uint16_t* out, int B, int nwg,
                          hipStream_t s);
enum { EPI_F32 = 0, EPI_F32_RELU = 1, EPI_T_GELU = 2, EPI_RESID = 3, EPI_PARTIAL = 4, EPI_T = 5 };
}  // namespace fac

namespace {

constexpr int kDim = 1024, kDepth = 6, kMlp = 2048, kPatchDim = 25088, kImg = 224;
constexpr float kBnEps = 1e-5f;

const int kStem[17][2] = {{3, 32},    {32, 32},   {32, 32},   {32, 64},   {64, 64},   {64, 64},
                          {64, 128},  {128, 128}, {128, 128}, {128, 256}, {256, 256}, {256, 256},
                          {256, 256}, {256, 512}, {512, 512}, {512, 512}, {512, 512}};
bool pool_after(int i) { return i == 2 || i == 5 || i == 8 || i == 12 || i == 16; }

struct ConvLayer {
  int H = 0, Cin = 0, Cout = 0;
  bool pool = false;
  uint16_t* w = nullptr;
  float* b = nullptr;
  // the 28^2 / 14^2 layers also packed for half the output-channel block
  // (bn_small), taken when the default grid leaves CUs idle (few crops: the
  // reference's one-video call); bit-identical outputs
  int bn_small = 0;
  uint16_t* w_small = nullptr;
  uint16_t* w_small32 = nullptr;  // the 14^2 layers packed for 32-channel blocks (option "conv_small14")
};

struct TLayer {
  float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
  uint16_t *wqkv = nullptr, *wo = nullptr, *w1 = nullptr, *w2 = nullptr;
  float *bo = nullptr, *b1 = nullptr, *b2 = nullptr;
};

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

struct fac_ctx {
  int device = 0;
  int dtype = 0;
  bool loaded = false;
  bool tail_only = false;  // option "tail_only": load/run only patch embedding .. head (ResVitKan)
  std::string err;
  std::vector<void*> weights;  // all weight allocations
  uint16_t* conv1_w = nullptr;
  uint16_t* conv1_wp = nullptr;  // conv1 weights in stem224's pixel-pair K order
  float* conv1_b = nullptr;
  ConvLayer conv[16];
  uint16_t* pe_w = nullptr;
  float *pe_b = nullptr, *cls = nullptr, *pos = nullptr;
  TLayer tl[kDepth];
  uint16_t* h1_w = nullptr;
  float *h1_b = nullptr, *h2_w = nullptr, *h2_b = nullptr;
  // workspace
  void* ws = nullptr;
  size_t ws_bytes = 0;
  int cap_B = 0;
  int stem_chunk = 0;
  int fuse_stem224 = 1;  // conv1..conv3+pool as one persistent kernel (stem224.hip)
  // GEMM tile variant per call site (transformer.hip launch_gemm; -1 = default)
  // and the split-K factor of the two N=1024 projections (to_out, FF2)
  int gemm_var[6] = {-1, -1, -1, -1, -1, -1};  // patch, qkv, out, ff1, ff2, head
  int proj_splits = 4;
  // software pipeline across batches (fac_forward_nhwc_u8_pipelined): batch k's
  // conv stack writes stem buffer k&1 on the caller's stream; its encoder +
  // head run on tail_st, ordered by ev_conv[k&1] / ev_tail[k&1]
  hipStream_t tail_st = nullptr;
  hipEvent_t ev_conv[2] = {nullptr, nullptr}, ev_tail[2] = {nullptr, nullptr};
  bool tail_pending[2] = {false, false};
  int pipe_k = 0;
  int tail_priority = 1;  // option "tail_priority": 1 = high-priority tail stream
  float ffn_ln_eps = 1e-5f;  // option "ffn_ln_eps_exp" n: eps = 10^-n of the FeedForward PreNorm LayerNorm
                             // (1e-6 in the RepBn8 variant's LinearNorm, cvit_GGCA_ADD_DEConv_RepBn8.py:48)
  uint16_t* stem_out2 = nullptr;
  int num_cu = 256;
  uint16_t *act0 = nullptr, *act1 = nullptr, *deep0 = nullptr, *deep1 = nullptr, *stem_out = nullptr, *xn = nullptr,
           *o = nullptr, *hbuf = nullptr, *cbuf = nullptr;
  int cap_chunk = 0;  // crops act0/act1 hold
  float *slab = nullptr, *x = nullptr, *qkv = nullptr, *hh = nullptr;
  // pos_index range flag: host-visible pinned memory (hipHostMalloc, mapped),
  // written by embed_finalize_ln with a plain system-scope store, read by the
  // host at the start of the next forward without a device sync
  int* errflag = nullptr;      // device view
  int* err_host = nullptr;     // host view of the same int
  // encoder launches on this context (the flag holds the offending one's
  // number).  It counts tail launches, not API calls: a pipelined or chunked
  // call counts once per batch, and a captured graph (the small-batch replay
  // or a caller's capture) bakes in the number of its capture, which every
  // replay then reports.
  int fwd_seq = 0;
  int stem_nwg = 0;      // option "stem_nwg": persistent stem workgroups (0 = one per CU)
  // option "stem_events": hipEvent pairs around every fused-stem launch (the
  // bench's timed region), read back by fac_stem_event_ms
  bool stem_ev = false;
  std::vector<hipEvent_t> stem_evs;
  size_t stem_ev_used = 0;
  uint16_t* zero16 = nullptr;  // 256 zero bytes: the source of zero-padding glds pieces
  // Forwards of one context share the activation and encoder buffers, so two
  // of them must never overlap on the device: every forward records ev_stack
  // on its stream after its last kernel (a synchronous forward: after the
  // head; a pipelined one: after its conv stack, its tail being ordered by
  // ev_tail), and a forward enqueued on a different stream first waits for
  // it.  Threads that share a context therefore need no common stream.
  // (Inside a stream capture the caller orders the graph launches; no
  // external event is waited on there.)
  hipEvent_t ev_stack = nullptr;
  hipStream_t stack_st = nullptr;
  bool stack_rec = false;
  // Small-batch graph replay (option "graph_max_b"): a forward of B <= this
  // many crops on a stream that is not being captured replays a hipGraph of
  // the whole forward, captured once per (B, input kind, probs) on cap_st
  // over context-owned input / slot / output buffers (g_in_*, g_pidx,
  // g_out).  The reference scores a video as ONE <= 29-crop call
  // (cvit_prediction.py:224-229), whose ~60 kernels are latency-bound at
  // that size: the graph turns them into one launch.
  struct SmallGraph {
    int B, kind;  // kind: bit 0 = uint8 NHWC input, bit 1 = probs wanted
    hipGraphExec_t exec;
    // direct graphs: captured on the caller's own buffers (no copies in or
    // out); nullptr in = the copy graph of (B, kind), over g_in / g_out
    const void* in = nullptr;
    const int32_t* pidx = nullptr;
    float *logits = nullptr, *probs = nullptr;
    unsigned long long used = 0;
  };
  // the previous small forward's buffers per (B, kind): a second call on the
  // same buffers captures a direct graph for them
  struct LastCall {
    int B, kind;
    const void* in;
    const int32_t* pidx;
    float *logits, *probs;
  };
  std::vector<LastCall> last_calls;
  unsigned long long graph_clock = 0;
  unsigned knob_gen = 0;  // g_knob_gen when this context's graphs were (last) known current
  static constexpr int kDirectGraphs = 8;
  int graph_max_b = 32;
  int conv_small = 1;  // option "conv_small": 28^2 / 14^2 layers on half-width column blocks when few crops
  int small14 = 1;  // option "conv_small14": few-crop 14^2 convs on 32-channel blocks when they fit one per CU (1) or never (0)
  std::vector<SmallGraph> graphs;
  hipStream_t cap_st = nullptr;
  void* g_in[2] = {nullptr, nullptr};  // [0] fp32 NCHW, [1] uint8 NHWC; graph_max_b crops each
  int32_t* g_pidx = nullptr;
  float* g_out = nullptr;  // logits [graph_max_b][2], then probs [graph_max_b][2]
  int g_cap = 0;           // crops the g_* buffers hold
};

namespace {

// Bumped by every fac_set_option call: several knobs are process-wide (they
// pick kernels for every context), so a graph another context captured before
// the change would keep the old kernels; forward_graph drops its context's
// graphs when the generation moved.  Graphs a caller captured
// around fac_* calls itself (torch.cuda.graph) are the caller's to recapture.
std::atomic<unsigned> g_knob_gen{0};

int set_err(fac_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// FAC_ERR_ARG if an earlier forward of this context saw a pos_index outside
// [0,32) (the device clamps it and raises the flag; the flag is read here,
// on the host, at the next call — no synchronisation)
int take_device_error(fac_ctx* c) {
  if (c && c->err_host && *(volatile int*)c->err_host) {
    const int bad = *(volatile int*)c->err_host;
    *(volatile int*)c->err_host = 0;
    return set_err(c, FAC_ERR_ARG, "encoder launch #" + std::to_string(bad) + " of this context (the next is #" +
                                       std::to_string(c->fwd_seq + 1) +
                                       "; graph replays report their capture's number) had a pos_index outside "
                                       "[0,32), clamped on the device; this call was not run");
  }
  return 0;
}

#define HIP_TRY(ctx, expr)                                                                  \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return set_err(ctx, FAC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

uint16_t to16(int dtype, float f) { return dtype == 0 ? fac_host::f32_to_bf16(f) : fac_host::f32_to_f16(f); }

// Split-K factor of the patch embedding (K = 25088 = 392 k-tiles of 64).  Fixed,
// so a crop's logits are bit-identical whatever batch it is scored in.
constexpr int kPatchSplits = 14;
constexpr int kProjSplitsMax = 4;  // split-K of the to_out / FF2 projections (fac_ctx::proj_splits)
int patch_splits(int) { return kPatchSplits; }

hipError_t run_conv(const fac_ctx* c, const ConvLayer& L, const uint16_t* in, uint16_t* out, int B, hipStream_t st) {
  using namespace fac;
  // the 14^2 layers on 32-channel blocks while that grid still fits one
  // workgroup per CU (B <= 16 crops for cout 512): at B = 1 / 8 the graph
  // forward 0.438 / 0.484 -> 0.419 / 0.465 ms; at B = 29 (464 workgroups)
  // the 64-channel blocks stay faster (0.655-0.669 vs 0.666-0.676 ms)
  if (L.w_small32 && c->conv_small && c->small14 && (long long)B * (L.Cout / 32) <= c->num_cu)
    return launch_conv3x3(c->dtype, in, L.w_small32, L.b, out, B, L.H, L.H, L.Cin, L.Cout, L.pool, c->zero16, st, true,
                          32);
  if (L.w_small && c->conv_small) {
    const int bn = conv_block_n(L.H, L.Cout), boxes = L.H == 14 ? 1 : (L.H / 4) * (L.H / 28);
    if ((long long)B * boxes * (L.Cout / bn) < c->num_cu)
      return launch_conv3x3(c->dtype, in, L.w_small, L.b, out, B, L.H, L.H, L.Cin, L.Cout, L.pool, c->zero16, st, true,
                            L.bn_small);
  }
  return launch_conv3x3(c->dtype, in, L.w, L.b, out, B, L.H, L.H, L.Cin, L.Cout, L.pool, c->zero16, st);
}

struct WsLayout {
  size_t act, deep, stem, stem2, slab, x, xn, qkv, o, hbuf, cbuf, hh, err, zero, total;
  int cb;  // crops the high-res activation buffers hold (stem chunk)
};

// Elements per crop of the largest activation each buffer pair holds:
// high-res stage (conv1..conv9, chunked): 224x224x32; deep stage (conv10..
// conv17, whole batch): 28x28x256.
constexpr size_t kActElems = (size_t)kImg * kImg * 32;
constexpr size_t kDeepElems = (size_t)28 * 28 * 256;
constexpr int kLastChunked = 7;  // c->conv[7] = conv9: the last conv run per stem chunk

WsLayout layout(int B, int chunk) {
  auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
  WsLayout L{};
  const int cb = (chunk > 0 && chunk < B) ? chunk : B;
  L.cb = cb;
  const size_t S = (size_t)std::max(kPatchSplits, 2 * kProjSplitsMax) * B;
  size_t off = 0;
  L.act = off; off += 2 * al((size_t)cb * kActElems * 2);
  L.deep = off; off += 2 * al((size_t)B * kDeepElems * 2);
  L.stem = off; off += al((size_t)B * kPatchDim * 2);
  L.stem2 = off; off += al((size_t)B * kPatchDim * 2);
  L.slab = off; off += al(S * kDim * 4);
  L.x = off; off += al((size_t)2 * B * kDim * 4);
  L.xn = off; off += al((size_t)2 * B * kDim * 2);
  L.qkv = off; off += al((size_t)2 * B * 3 * kDim * 4);
  L.o = off; off += al((size_t)2 * B * kDim * 2);
  L.hbuf = off; off += al((size_t)2 * B * kMlp * 2);
  L.cbuf = off; off += al((size_t)B * kDim * 2);
  L.hh = off; off += al((size_t)B * kMlp * 4);
  L.err = off; off += 256;
  L.zero = off; off += 256;
  L.total = off;
  return L;
}

// Drop the captured small-batch graphs (they hold the workspace and weight
// pointers and the kernel choices of the options they were captured with):
// on a workspace reallocation, a weight load, an option change or destroy.
void drop_graphs(fac_ctx* c) {
  if (c->graphs.empty()) return;
  (void)hipDeviceSynchronize();  // no replay of them is still in flight
  for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.exec);
  c->graphs.clear();
  c->last_calls.clear();
}

int ensure_ws(fac_ctx* c, int B) {
  if (B <= c->cap_B && c->ws) return FAC_OK;
  drop_graphs(c);
  const WsLayout L = layout(B, c->stem_chunk);
  if (c->ws) {
    HIP_TRY(c, hipDeviceSynchronize());
    HIP_TRY(c, hipFree(c->ws));
    c->ws = nullptr;
  }
  if (hipMalloc(&c->ws, L.total) != hipSuccess) {
    c->ws = nullptr;
    c->cap_B = 0;
    return set_err(c, FAC_ERR_OOM, "workspace allocation of " + std::to_string(L.total) + " bytes failed");
  }
  HIP_TRY(c, hipMemset(c->ws, 0, L.total));
  char* base = (char*)c->ws;
  const size_t half = (L.deep - L.act) / 2, dhalf = (L.stem - L.deep) / 2;
  c->act0 = (uint16_t*)(base + L.act);
  c->act1 = (uint16_t*)(base + L.act + half);
  c->deep0 = (uint16_t*)(base + L.deep);
  c->deep1 = (uint16_t*)(base + L.deep + dhalf);
  c->cap_chunk = L.cb;
  c->stem_out = (uint16_t*)(base + L.stem);
  c->stem_out2 = (uint16_t*)(base + L.stem2);
  c->slab = (float*)(base + L.slab);
  c->x = (float*)(base + L.x);
  c->xn = (uint16_t*)(base + L.xn);
  c->qkv = (float*)(base + L.qkv);
  c->o = (uint16_t*)(base + L.o);
  c->hbuf = (uint16_t*)(base + L.hbuf);
  c->cbuf = (uint16_t*)(base + L.cbuf);
  c->hh = (float*)(base + L.hh);
  if (!c->err_host) {
    void* hp = nullptr;
    HIP_TRY(c, hipHostMalloc(&hp, 256, hipHostMallocMapped | hipHostMallocCoherent));
    c->err_host = (int*)hp;
    *(volatile int*)c->err_host = 0;
    void* dp = nullptr;
    HIP_TRY(c, hipHostGetDevicePointer(&dp, hp, 0));
    c->errflag = (int*)dp;
  }
  c->zero16 = (uint16_t*)(base + L.zero);  // the whole workspace was just zeroed
  c->ws_bytes = L.total;
  c->cap_B = B;
  return FAC_OK;
}

template <class U>
int upload(fac_ctx* c, const std::vector<U>& host, U** dst) {
  void* p = nullptr;
  if (hipMalloc(&p, host.size() * sizeof(U)) != hipSuccess) return set_err(c, FAC_ERR_OOM, "weight allocation failed");
  c->weights.push_back(p);
  HIP_TRY(c, hipMemcpy(p, host.data(), host.size() * sizeof(U), hipMemcpyHostToDevice));
  *dst = (U*)p;
  return FAC_OK;
}

struct Descs {
  std::map<std::string, const fac_tensor_desc*> m;
  fac_ctx* c;
  std::string missing;
  const float* get(const std::string& name, std::initializer_list<int64_t> shape, int* rc) {
    auto it = m.find(name);
    if (it == m.end()) {
      *rc = set_err(c, FAC_ERR_MISSING, "missing state_dict key: " + name);
      return nullptr;
    }
    const fac_tensor_desc* d = it->second;
    std::vector<int64_t> want(shape);
    bool ok = d->data != nullptr && d->ndim == (int)want.size();
    for (size_t i = 0; ok && i < want.size(); ++i) ok = d->shape[i] == want[i];
    if (!ok) {
      std::string got;
      for (int i = 0; i < d->ndim && i < 4; ++i) got += std::to_string(d->shape[i]) + ",";
      *rc = set_err(c, FAC_ERR_SHAPE, "shape mismatch for " + name + " (got [" + got + "])");
      return nullptr;
    }
    return d->data;
  }
};

std::vector<uint16_t> convert16(int dtype, const float* src, size_t n) {
  std::vector<uint16_t> out(n);
  for (size_t i = 0; i < n; ++i) out[i] = to16(dtype, src[i]);
  return out;
}

// nn.Sequential indices of conv i and its BatchNorm (cvit.py:86-148).
void stem_indices(int i, int* cidx, int* bidx) {
  int idx = 0;
  for (int k = 0; k < i; ++k) idx += 3 + (pool_after(k) ? 1 : 0);
  *cidx = idx;
  *bidx = idx + 1;
}

int load_impl(fac_ctx* c, const fac_tensor_desc* descs, int n) {
  Descs D{{}, c, {}};
  for (int i = 0; i < n; ++i) {
    if (!descs[i].name) return set_err(c, FAC_ERR_ARG, "descriptor with null name");
    D.m[descs[i].name] = &descs[i];
  }
  int rc = FAC_OK;
#define GET(var, name, ...)                                 \
  const float* var = D.get(name, {__VA_ARGS__}, &rc);       \
  if (!var) return rc;

  // ---- conv stem with BN folded
  int H = kImg;
  for (int i = 0; i < 17 && !c->tail_only; ++i) {
    const int ci = kStem[i][0], co = kStem[i][1];
    int cidx, bidx;
    stem_indices(i, &cidx, &bidx);
    const std::string pc = "features." + std::to_string(cidx) + ".", pb = "features." + std::to_string(bidx) + ".";
    GET(w, pc + "weight", co, ci, 3, 3);
    GET(bconv, pc + "bias", co);
    GET(gam, pb + "weight", co);
    GET(bet, pb + "bias", co);
    GET(mean, pb + "running_mean", co);
    GET(var, pb + "running_var", co);
    std::vector<float> s(co), bf(co);
    for (int o = 0; o < co; ++o) {
      s[o] = gam[o] / std::sqrt(var[o] + kBnEps);
      bf[o] = (bconv[o] - mean[o]) * s[o] + bet[o];
    }
    auto wf = [&](int o, int cin, int t) { return w[((size_t)o * ci + cin) * 9 + t] * s[o]; };
    std::vector<float> wfold((size_t)co * ci * 9);  // BN-folded fp32 [co][ci][9]
    for (int o = 0; o < co; ++o)
      for (int cin = 0; cin < ci; ++cin)
        for (int t = 0; t < 9; ++t) wfold[((size_t)o * ci + cin) * 9 + t] = wf(o, cin, t);
    if (i == 0) {
      std::vector<uint16_t> pk((size_t)32 * 64, 0);
      for (int o = 0; o < 32; ++o)
        for (int t = 0; t < 9; ++t)
          for (int cin = 0; cin < 3; ++cin) pk[(size_t)o * 64 + t * 4 + cin] = to16(c->dtype, wf(o, cin, t));
      if ((rc = upload(c, pk, &c->conv1_w))) return rc;
      std::vector<uint16_t> pp((size_t)32 * 64);
      fac::pack_stem_conv1(c->dtype, wfold.data(), pp.data());  // stem224's pixel-pair K order (stack_ops.hip)
      if ((rc = upload(c, pp, &c->conv1_wp))) return rc;
      if ((rc = upload(c, bf, &c->conv1_b))) return rc;
    } else {
      ConvLayer& L = c->conv[i - 1];
      L.H = H;
      L.Cin = ci;
      L.Cout = co;
      L.pool = pool_after(i);
      std::vector<uint16_t> pk((size_t)co * ci * 9);
      fac::pack_conv3x3(c->dtype, H, ci, co, wfold.data(), pk.data());  // the LDS-image order of conv.hip
      if ((rc = upload(c, pk, &L.w))) return rc;
      L.bn_small = H == 14 ? 64 : (H == 28 ? 128 : 0);
      L.w_small = nullptr;
      if (L.bn_small) {
        fac::pack_conv3x3(c->dtype, H, ci, co, wfold.data(), pk.data(), L.bn_small);
        if ((rc = upload(c, pk, &L.w_small))) return rc;
      }
      L.w_small32 = nullptr;
      if (H == 14) {
        fac::pack_conv3x3(c->dtype, H, ci, co, wfold.data(), pk.data(), 32);
        if ((rc = upload(c, pk, &L.w_small32))) return rc;
      }
      if ((rc = upload(c, bf, &L.b))) return rc;
    }
    if (pool_after(i)) H /= 2;
  }

  // ---- embeddings
  GET(pos, "pos_embedding", 32, 1, kDim);
  GET(cls, "cls_token", 1, 1, kDim);
  GET(pew, "patch_to_embedding.weight", kDim, kPatchDim);
  GET(peb, "patch_to_embedding.bias", kDim);
  if ((rc = upload(c, std::vector<float>(pos, pos + 32 * kDim), &c->pos))) return rc;
  if ((rc = upload(c, std::vector<float>(cls, cls + kDim), &c->cls))) return rc;
  if ((rc = upload(c, convert16(c->dtype, pew, (size_t)kDim * kPatchDim), &c->pe_w))) return rc;
  if ((rc = upload(c, std::vector<float>(peb, peb + kDim), &c->pe_b))) return rc;

  // ---- transformer (cvit.py:64-78; key layout transformer.layers.{l}.{0,1}.fn.{norm,fn}.*)
  for (int l = 0; l < kDepth; ++l) {
    const std::string p = "transformer.layers." + std::to_string(l) + ".";
    TLayer& T = c->tl[l];
    GET(g1, p + "0.fn.norm.weight", kDim);
    GET(b1n, p + "0.fn.norm.bias", kDim);
    GET(wqkv, p + "0.fn.fn.to_qkv.weight", 3 * kDim, kDim);
    GET(wo, p + "0.fn.fn.to_out.weight", kDim, kDim);
    GET(bo, p + "0.fn.fn.to_out.bias", kDim);
    GET(g2, p + "1.fn.norm.weight", kDim);
    GET(b2n, p + "1.fn.norm.bias", kDim);
    GET(w1, p + "1.fn.fn.net.0.weight", kMlp, kDim);
    GET(b1, p + "1.fn.fn.net.0.bias", kMlp);
    GET(w2, p + "1.fn.fn.net.2.weight", kDim, kMlp);
    GET(b2, p + "1.fn.fn.net.2.bias", kDim);
    if ((rc = upload(c, std::vector<float>(g1, g1 + kDim), &T.ln1_g))) return rc;
    if ((rc = upload(c, std::vector<float>(b1n, b1n + kDim), &T.ln1_b))) return rc;
    if ((rc = upload(c, std::vector<float>(g2, g2 + kDim), &T.ln2_g))) return rc;
    if ((rc = upload(c, std::vector<float>(b2n, b2n + kDim), &T.ln2_b))) return rc;
    if ((rc = upload(c, convert16(c->dtype, wqkv, (size_t)3 * kDim * kDim), &T.wqkv))) return rc;
    if ((rc = upload(c, convert16(c->dtype, wo, (size_t)kDim * kDim), &T.wo))) return rc;
    if ((rc = upload(c, std::vector<float>(bo, bo + kDim), &T.bo))) return rc;
    if ((rc = upload(c, convert16(c->dtype, w1, (size_t)kMlp * kDim), &T.w1))) return rc;
    if ((rc = upload(c, std::vector<float>(b1, b1 + kMlp), &T.b1))) return rc;
    if ((rc = upload(c, convert16(c->dtype, w2, (size_t)kDim * kMlp), &T.w2))) return rc;
    if ((rc = upload(c, std::vector<float>(b2, b2 + kDim), &T.b2))) return rc;
  }

  // ---- head (cvit.py:161-165)
  GET(h1w, "mlp_head.0.weight", kMlp, kDim);
  GET(h1b, "mlp_head.0.bias", kMlp);
  GET(h2w, "mlp_head.2.weight", 2, kMlp);
  GET(h2b, "mlp_head.2.bias", 2);
  if ((rc = upload(c, convert16(c->dtype, h1w, (size_t)kMlp * kDim), &c->h1_w))) return rc;
  if ((rc = upload(c, std::vector<float>(h1b, h1b + kMlp), &c->h1_b))) return rc;
  if ((rc = upload(c, std::vector<float>(h2w, h2w + 2 * kMlp), &c->h2_w))) return rc;
  if ((rc = upload(c, std::vector<float>(h2b, h2b + 2), &c->h2_b))) return rc;
#undef GET
  c->loaded = true;
  return FAC_OK;
}

// Optional per-stage event timing (fac_profile_forward_u8): an event after
// every stage, tagged with the stage id; durations are summed per stage over
// stem chunks.  stop_after >= 0 (fac_debug_features_u8) copies conv
// `stop_after`'s output to feat_out and returns.
struct Prof {
  std::vector<hipEvent_t> ev;
  std::vector<int> stage;
};

int tail_impl(fac_ctx* c, const uint16_t* stem, int B, const int32_t* pidx, float* logits, float* probs,
              hipStream_t st, Prof* prof, float* hidden_out = nullptr, bool beside_stack = false);

// The synchronous forward on `stream`: conv stack -> stem_dst (default the
// context's stem buffer 0), then (unless conv_only) the encoder and head.
int forward_impl(fac_ctx* c, const void* in, bool u8, int B, const int32_t* pidx, float* logits, float* probs,
                 void* stream, Prof* prof = nullptr, int stop_after = -1, uint16_t* feat_out = nullptr,
                 const uint16_t* stem_in = nullptr, uint16_t* stem_dst = nullptr, bool conv_only = false) {
  using namespace fac;
  if (!c) return FAC_ERR_ARG;
  if (!c->loaded) return set_err(c, FAC_ERR_NOT_LOADED, "forward before fac_load_weights");
  if (c->tail_only && !stem_in)
    return set_err(c, FAC_ERR_NOT_LOADED, "tail-only context has no conv stem: use fac_forward_features");
  if (B <= 0 || (!in && !stem_in) || (stop_after < 0 && !conv_only && (!pidx || !logits)))
    return set_err(c, FAC_ERR_ARG, "bad forward arguments");
  if (int e = take_device_error(c)) return e;
  DevGuard g(c->device);
  int rc = ensure_ws(c, B);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  // order this conv stack after the context's previous one (see fac_ctx::ev_stack)
  struct StackOrder {
    fac_ctx* c;
    hipStream_t st;
    bool active;
    ~StackOrder() {
      if (active && hipEventRecord(c->ev_stack, st) == hipSuccess) {
        c->stack_st = st;
        c->stack_rec = true;
      }
    }
  } order{c, st, false};
  if (!stem_in) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(c, hipStreamIsCapturing(st, &cs));
    if (cs == hipStreamCaptureStatusNone) {
      if (!c->ev_stack) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_stack, hipEventDisableTiming));
      if (c->stack_rec && c->stack_st != st) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_stack, 0));
      order.active = true;
    }
  }
  if (!stem_dst) {
    // a synchronous forward shares the encoder workspace with pipelined
    // tails still in flight: order it after them
    stem_dst = c->stem_out;
    for (int i = 0; i < 2; ++i)
      if (c->tail_pending[i]) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_tail[i], 0));
  }
  const int dt = c->dtype;
  const int chunk = std::min(B, c->cap_chunk);
#define MARK(sid)                                  \
  do {                                             \
    if (prof) {                                    \
      hipEvent_t mk_;                              \
      HIP_TRY(c, hipEventCreate(&mk_));            \
      prof->ev.push_back(mk_);                     \
      prof->stage.push_back(sid);                  \
      HIP_TRY(c, hipEventRecord(mk_, st));         \
    }                                              \
  } while (0)
  auto conv_out_elems = [](const ConvLayer& L) {  // per crop
    const size_t Ho = L.pool ? L.H / 2 : L.H;
    return Ho * Ho * (size_t)L.Cout;
  };
  MARK(-1);
  // Stage A, per stem chunk (a sub-batch whose high-res activations can stay
  // in the Infinity Cache): conv1..conv9, output pooled 28x28x128 into the
  // whole-batch deep buffer.
  for (int b0 = 0; b0 < B && !stem_in; b0 += chunk) {
    const int nb = std::min(chunk, B - b0);
    if (nb > c->cap_chunk) return set_err(c, FAC_ERR_ARG, "internal: stem chunk exceeds workspace");
    const void* src = u8 ? (const void*)((const uint8_t*)in + (size_t)b0 * kImg * kImg * 3)
                         : (const void*)((const float*)in + (size_t)b0 * 3 * kImg * kImg);
    uint16_t *cur = c->act0, *nxt = c->act1;
    int l0 = 0;
    bool copied = false;  // stop_after's output already copied for this chunk
    if (c->fuse_stem224 && (stop_after < 0 || stop_after >= 2)) {
      // conv1..conv3 + pool in one kernel; the profile reports it as stage 0 (conv1)
      hipEvent_t sev0 = nullptr, sev1 = nullptr;
      if (c->stem_ev) {
        while (c->stem_evs.size() < c->stem_ev_used + 2) {
          hipEvent_t e;
          HIP_TRY(c, hipEventCreate(&e));
          c->stem_evs.push_back(e);
        }
        sev0 = c->stem_evs[c->stem_ev_used];
        sev1 = c->stem_evs[c->stem_ev_used + 1];
        c->stem_ev_used += 2;
        HIP_TRY(c, hipEventRecord(sev0, st));
      }
      HIP_TRY(c, launch_stem224(dt, u8, src, c->conv1_wp, c->conv1_b, c->conv[0].w, c->conv[0].b, c->conv[1].w,
                                c->conv[1].b, cur, nb, c->stem_nwg > 0 ? c->stem_nwg : c->num_cu, st));
      if (sev1) HIP_TRY(c, hipEventRecord(sev1, st));
      MARK(0);
      l0 = 2;
      if (stop_after == 2) {
        HIP_TRY(c, hipMemcpyAsync(feat_out + (size_t)b0 * conv_out_elems(c->conv[1]), cur,
                                  (size_t)nb * conv_out_elems(c->conv[1]) * 2, hipMemcpyDeviceToDevice, st));
        copied = true;
      }
    } else {
      HIP_TRY(c, launch_conv1(dt, u8, src, c->conv1_w, c->conv1_b, cur, nb, kImg, kImg, st));
      MARK(0);
      if (stop_after == 0) {
        HIP_TRY(c, hipMemcpyAsync(feat_out + (size_t)b0 * kActElems, cur, (size_t)nb * kActElems * 2,
                                  hipMemcpyDeviceToDevice, st));
        copied = true;
      }
    }
    for (int l = l0; l <= kLastChunked && !copied; ++l) {
      const ConvLayer& L = c->conv[l];
      uint16_t* dst = (l == kLastChunked) ? c->deep0 + (size_t)b0 * conv_out_elems(L) : nxt;
      HIP_TRY(c, run_conv(c, L, cur, dst, nb, st));
      MARK(l + 1);
      if (stop_after == l + 1 && l != kLastChunked) {
        HIP_TRY(c, hipMemcpyAsync(feat_out + (size_t)b0 * conv_out_elems(L), dst, (size_t)nb * conv_out_elems(L) * 2,
                                  hipMemcpyDeviceToDevice, st));
        copied = true;
      }
      std::swap(cur, nxt);
    }
  }
  if (stop_after >= 0 && stop_after <= kLastChunked) return FAC_OK;  // copied per chunk above
  // Stage B, whole batch: conv10..conv17 -> stem_out [B,7,7,512].
  if (!stem_in) {
    uint16_t *cur = c->deep0, *nxt = c->deep1;
    if (stop_after == kLastChunked + 1) {
      HIP_TRY(c, hipMemcpyAsync(feat_out, cur, (size_t)B * conv_out_elems(c->conv[kLastChunked]) * 2,
                                hipMemcpyDeviceToDevice, st));
      return FAC_OK;
    }
    for (int l = kLastChunked + 1; l < 16; ++l) {
      const ConvLayer& L = c->conv[l];
      uint16_t* dst = (l == 15) ? stem_dst : nxt;
      HIP_TRY(c, run_conv(c, L, cur, dst, B, st));
      MARK(l + 1);
      if (stop_after == l + 1) {
        HIP_TRY(c, hipMemcpyAsync(feat_out, dst, (size_t)B * conv_out_elems(L) * 2, hipMemcpyDeviceToDevice, st));
        return FAC_OK;
      }
      std::swap(cur, nxt);
    }
  }
  if (conv_only) return FAC_OK;
  return tail_impl(c, stem_in ? stem_in : stem_dst, B, pidx, logits, probs, st, prof);
#undef MARK
}

// Patch embedding, the 6 encoder layers and the head on `st`, from the conv
// stack's output `stem` [B,7,7,512] (cvit.py:171-179).
int tail_impl(fac_ctx* c, const uint16_t* stem, int B, const int32_t* pidx, float* logits, float* probs,
              hipStream_t st, Prof* prof, float* hidden_out, bool beside_stack) {
  using namespace fac;
  const int dt = c->dtype;
  // beside_stack: this encoder co-runs with the next batch's conv stack (the
  // pipelined forward): the default tile rule for that case (launch_gemm, -2)
  int gv[6];
  for (int i = 0; i < 6; ++i) gv[i] = (beside_stack && c->gemm_var[i] == -1) ? -2 : c->gemm_var[i];
#define MARK(sid)                                  \
  do {                                             \
    if (prof) {                                    \
      hipEvent_t mk_;                              \
      HIP_TRY(c, hipEventCreate(&mk_));            \
      prof->ev.push_back(mk_);                     \
      prof->stage.push_back(sid);                  \
      HIP_TRY(c, hipEventRecord(mk_, st));         \
    }                                              \
  } while (0)
  const int S = patch_splits(B);
  HIP_TRY(c, launch_gemm(dt, EPI_PARTIAL, stem, kPatchDim, c->pe_w, kPatchDim, nullptr, c->slab, kDim, B, kDim,
                         kPatchDim, S, st, gv[0]));
  // residual stream rows + layer 0's PreNorm LayerNorm in one pass
  HIP_TRY(c, launch_embed_finalize_ln(dt, c->slab, S, B, c->pe_b, c->cls, c->pos, pidx, c->x, c->tl[0].ln1_g,
                                      c->tl[0].ln1_b, c->xn, c->errflag, ++c->fwd_seq, st));
  MARK(17);
  const int R = 2 * B;
  const float scale = 1.0f / std::sqrt((float)kDim);  // dim ** -0.5 (cvit.py:38), not head_dim
  // The two N=1024 projections (to_out, FF2) run split-K into fp32 partial
  // slabs; the following kernel (residual add + next LayerNorm, or the CLS
  // finish after the last layer) sums them in split order.
  const int SK = c->proj_splits;
  for (int l = 0; l < kDepth; ++l) {
    const TLayer& T = c->tl[l];
    if (l > 0) {
      HIP_TRY(c, launch_resid_layernorm(dt, c->x, c->slab, SK, c->tl[l - 1].b2, T.ln1_g, T.ln1_b, c->xn, R, st));
    }
    HIP_TRY(c, launch_gemm(dt, EPI_F32, c->xn, kDim, T.wqkv, kDim, nullptr, c->qkv, 3 * kDim, R, 3 * kDim, kDim, 1, st,
                           gv[1]));
    HIP_TRY(c, launch_attention2(dt, c->qkv, c->o, B, scale, st));
    HIP_TRY(c, launch_gemm(dt, EPI_PARTIAL, c->o, kDim, T.wo, kDim, nullptr, c->slab, kDim, R, kDim, kDim, SK, st,
                           gv[2]));
    HIP_TRY(c, launch_resid_layernorm(dt, c->x, c->slab, SK, T.bo, T.ln2_g, T.ln2_b, c->xn, R, st, c->ffn_ln_eps));
    HIP_TRY(c, launch_gemm(dt, EPI_T_GELU, c->xn, kDim, T.w1, kDim, T.b1, c->hbuf, kMlp, R, kMlp, kDim, 1, st,
                           gv[3]));
    HIP_TRY(c, launch_gemm(dt, EPI_PARTIAL, c->hbuf, kMlp, T.w2, kMlp, nullptr, c->slab, kDim, R, kDim, kMlp, SK, st, gv[4]));
  }
  MARK(18);
  HIP_TRY(c, launch_resid_cls(dt, c->x, c->slab, SK, c->tl[kDepth - 1].b2, c->cbuf, B, st));
  // hidden_out: the ReLU'd first head layer is the result (ResVitKan's KAN head follows)
  float* hh = hidden_out ? hidden_out : c->hh;
  HIP_TRY(c, launch_gemm(dt, EPI_F32_RELU, c->cbuf, kDim, c->h1_w, kDim, c->h1_b, hh, kMlp, B, kMlp, kDim, 1, st,
                         gv[5]));
  if (logits) HIP_TRY(c, launch_head_out(hh, c->h2_w, c->h2_b, logits, probs, B, st));
  MARK(19);
#undef MARK
  return FAC_OK;
}

// Order work enqueued on `st` after the context's previous forward on another
// stream and after any pipelined tail still in flight (fac_ctx::ev_stack).
int order_on(fac_ctx* c, hipStream_t st) {
  if (!c->ev_stack) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_stack, hipEventDisableTiming));
  if (c->stack_rec && c->stack_st != st) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_stack, 0));
  for (int i = 0; i < 2; ++i)
    if (c->tail_pending[i]) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_tail[i], 0));
  return FAC_OK;
}

int mark_done(fac_ctx* c, hipStream_t st) {
  HIP_TRY(c, hipEventRecord(c->ev_stack, st));
  c->stack_st = st;
  c->stack_rec = true;
  return FAC_OK;
}

// Capture forward_impl(in, pidx, logits, probs) at B as a graph (on the
// context's capture stream: the captured forward must not wait on events
// recorded outside the capture; the replay's ordering is done on the
// caller's stream).
int capture_forward(fac_ctx* c, const void* in, bool u8, int B, const int32_t* pidx, float* logits, float* probs,
                    hipGraphExec_t* out) {
  if (!c->cap_st) HIP_TRY(c, hipStreamCreateWithFlags(&c->cap_st, hipStreamNonBlocking));
  const bool tp0 = c->tail_pending[0], tp1 = c->tail_pending[1];
  c->tail_pending[0] = c->tail_pending[1] = false;
  HIP_TRY(c, hipStreamBeginCapture(c->cap_st, hipStreamCaptureModeThreadLocal));
  const int rc = forward_impl(c, in, u8, B, pidx, logits, probs, c->cap_st);
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(c->cap_st, &graph);
  c->tail_pending[0] = tp0;
  c->tail_pending[1] = tp1;
  if (rc != FAC_OK || ec != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc != FAC_OK ? rc : set_err(c, FAC_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(ec));
  }
  const hipError_t ei = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ei != hipSuccess) return set_err(c, FAC_ERR_HIP, std::string("graph instantiate: ") + hipGetErrorString(ei));
  return FAC_OK;
}

// The small-batch forward by graph replay (fac_ctx::graphs).  A call on the
// same buffers (crops, slots, logits, probs) as the previous call of its
// (B, kind) replays a graph captured on those buffers -- one graph launch,
// nothing copied (the reference's per-video loop reuses its buffers: torch's
// caching allocator hands the same blocks back); otherwise the crops and
// slots are copied into the context's buffers, the (B, kind) copy graph runs
// and the logits (and probabilities) are copied out.  Every graph holds the
// same kernels with the same arguments as forward_impl at this B, so the
// outputs are bit-identical to the eager forward.
int forward_graph(fac_ctx* c, const void* in, bool u8, int B, const int32_t* pidx, float* logits, float* probs,
                  hipStream_t st) {
  if (int e = take_device_error(c)) return e;
  DevGuard g(c->device);
  int rc = ensure_ws(c, B);
  if (rc) return rc;
  if (const unsigned gen = g_knob_gen.load(); gen != c->knob_gen) {
    drop_graphs(c);  // a process-wide knob changed since these were captured
    c->knob_gen = gen;
  }
  const int kind = (u8 ? 1 : 0) | (probs ? 2 : 0);
  ++c->graph_clock;
  // direct graph for these buffers?
  for (auto& gr : c->graphs)
    if (gr.in && gr.B == B && gr.kind == kind && gr.in == in && gr.pidx == pidx && gr.logits == logits &&
        gr.probs == probs) {
      gr.used = c->graph_clock;
      rc = order_on(c, st);
      if (rc) return rc;
      HIP_TRY(c, hipGraphLaunch(gr.exec, st));
      return mark_done(c, st);
    }
  bool repeat = false, seen = false;
  for (auto& lc : c->last_calls)
    if (lc.B == B && lc.kind == kind) {
      repeat = lc.in == in && lc.pidx == pidx && lc.logits == logits && lc.probs == probs;
      lc = {B, kind, in, pidx, logits, probs};
      seen = true;
    }
  if (!seen) c->last_calls.push_back({B, kind, in, pidx, logits, probs});
  if (repeat) {
    int ndirect = 0;
    fac_ctx::SmallGraph* oldest = nullptr;
    for (auto& gr : c->graphs)
      if (gr.in) {
        ++ndirect;
        if (!oldest || gr.used < oldest->used) oldest = &gr;
      }
    if (ndirect >= fac_ctx::kDirectGraphs) {
      // no replay of it may still be in flight on any stream
      HIP_TRY(c, hipDeviceSynchronize());
      (void)hipGraphExecDestroy(oldest->exec);
      c->graphs.erase(c->graphs.begin() + (oldest - c->graphs.data()));
    }
    hipGraphExec_t ex = nullptr;
    rc = capture_forward(c, in, u8, B, pidx, logits, probs, &ex);
    if (rc) return rc;
    fac_ctx::SmallGraph sg{B, kind, ex};
    sg.in = in;
    sg.pidx = pidx;
    sg.logits = logits;
    sg.probs = probs;
    sg.used = c->graph_clock;
    c->graphs.push_back(sg);
    rc = order_on(c, st);
    if (rc) return rc;
    HIP_TRY(c, hipGraphLaunch(ex, st));
    return mark_done(c, st);
  }
  const size_t crop_bytes = u8 ? (size_t)kImg * kImg * 3 : (size_t)3 * kImg * kImg * 4;
  if (c->g_cap < c->graph_max_b) {
    drop_graphs(c);
    for (void*& p : c->g_in) {
      if (p) HIP_TRY(c, hipFree(p));
      p = nullptr;
    }
    if (c->g_pidx) HIP_TRY(c, hipFree(c->g_pidx));
    if (c->g_out) HIP_TRY(c, hipFree(c->g_out));
    c->g_pidx = nullptr;
    c->g_out = nullptr;
    c->g_cap = 0;
    if (hipMalloc(&c->g_pidx, (size_t)c->graph_max_b * 4) != hipSuccess ||
        hipMalloc(&c->g_out, (size_t)c->graph_max_b * 16) != hipSuccess)
      return set_err(c, FAC_ERR_OOM, "graph buffer allocation failed");
    HIP_TRY(c, hipMemset(c->g_pidx, 0, (size_t)c->graph_max_b * 4));
    c->g_cap = c->graph_max_b;
  }
  void*& gin = c->g_in[u8 ? 1 : 0];
  if (!gin && hipMalloc(&gin, (size_t)c->g_cap * crop_bytes) != hipSuccess) {
    gin = nullptr;
    return set_err(c, FAC_ERR_OOM, "graph input buffer allocation failed");
  }
  float* const g_probs = c->g_out + 2 * c->g_cap;
  hipGraphExec_t ex = nullptr;
  for (auto& gr : c->graphs)
    if (!gr.in && gr.B == B && gr.kind == kind) ex = gr.exec;
  if (!ex) {
    rc = capture_forward(c, gin, u8, B, c->g_pidx, c->g_out, probs ? g_probs : nullptr, &ex);
    if (rc) return rc;
    c->graphs.push_back({B, kind, ex});
  }
  rc = order_on(c, st);
  if (rc) return rc;
  HIP_TRY(c, hipMemcpyAsync(gin, in, (size_t)B * crop_bytes, hipMemcpyDeviceToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(c->g_pidx, pidx, (size_t)B * 4, hipMemcpyDeviceToDevice, st));
  HIP_TRY(c, hipGraphLaunch(ex, st));
  HIP_TRY(c, hipMemcpyAsync(logits, c->g_out, (size_t)B * 8, hipMemcpyDeviceToDevice, st));
  if (probs) HIP_TRY(c, hipMemcpyAsync(probs, g_probs, (size_t)B * 8, hipMemcpyDeviceToDevice, st));
  return mark_done(c, st);
}

// fac_forward_nchw_f32 / fac_forward_nhwc_u8: small batches on a stream that
// is not being captured replay a graph, everything else runs eagerly.
int forward_entry(fac_ctx* c, const void* in, bool u8, int B, const int32_t* pidx, float* logits, float* probs,
                  void* stream) {
  if (c && c->loaded && !c->tail_only && in && pidx && logits && B > 0 && B <= c->graph_max_b && !c->stem_ev) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    DevGuard g(c->device);
    HIP_TRY(c, hipStreamIsCapturing((hipStream_t)stream, &cs));
    if (cs == hipStreamCaptureStatusNone) return forward_graph(c, in, u8, B, pidx, logits, probs, (hipStream_t)stream);
  }
  return forward_impl(c, in, u8, B, pidx, logits, probs, stream);
}

}  // namespace

extern "C" {

int fac_create(int device, int dtype, fac_ctx** out) {
  if (!out || (dtype != FAC_DTYPE_BF16 && dtype != FAC_DTYPE_F16)) return FAC_ERR_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return FAC_ERR_HIP;
  fac_ctx* c = new fac_ctx();
  c->device = device;
  c->dtype = dtype;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    c->num_cu = ncu;
  *out = c;
  return FAC_OK;
}

int fac_load_weights(fac_ctx* c, const fac_tensor_desc* descs, int n) {
  if (!c || !descs || n <= 0) return set_err(c, FAC_ERR_ARG, "bad load arguments");
  DevGuard g(c->device);
  drop_graphs(c);
  for (void* p : c->weights) (void)hipFree(p);
  c->weights.clear();
  c->loaded = false;
  return load_impl(c, descs, n);
}

int fac_reserve(fac_ctx* c, int max_batch) {
  if (!c || max_batch <= 0) return set_err(c, FAC_ERR_ARG, "bad reserve arguments");
  DevGuard g(c->device);
  return ensure_ws(c, max_batch);
}

int fac_workspace_bytes(fac_ctx* c, int B, size_t* out) {
  if (!c || !out || B <= 0) return FAC_ERR_ARG;
  *out = layout(B, c->stem_chunk).total;
  return FAC_OK;
}

int fac_set_stem_chunk(fac_ctx* c, int crops) {
  if (!c || crops < 0) return FAC_ERR_ARG;
  if (crops != c->stem_chunk) {
    DevGuard g(c->device);
    drop_graphs(c);
    c->stem_chunk = crops;
    const int cap = c->cap_B;
    c->cap_B = 0;  // force re-layout on next use
    if (cap > 0) {
      DevGuard g(c->device);
      return ensure_ws(c, cap);
    }
  }
  return FAC_OK;
}

int fac_set_option(fac_ctx* c, const char* key, int value) {
  if (!c || !key) return FAC_ERR_ARG;
  const std::string k(key);
  {  // every knob can change what a captured forward would launch -- in this
     // context, and for the process-wide ones in every other (g_knob_gen)
    DevGuard g(c->device);
    drop_graphs(c);
    c->knob_gen = ++g_knob_gen;
  }
  if (k == "stem_chunk") return fac_set_stem_chunk(c, value);
  if (k == "conv_ring9") {  // process-wide A/B: 9-slice weight ring (bit 0: the 14x14 / BN 64 tile)
    if (value < 0 || value > 7) return set_err(c, FAC_ERR_ARG, "conv_ring9 must be 0..7");
    fac::set_conv_ring9(value);
    return FAC_OK;
  }
  if (k == "conv_small14") {
    c->small14 = value != 0;
    return FAC_OK;
  }
  if (k == "conv_small") {
    c->conv_small = value != 0;
    return FAC_OK;
  }
  if (k == "graph_max_b") {
    if (value < 0 || value > 256) return set_err(c, FAC_ERR_ARG, "graph_max_b must be 0..256");
    c->graph_max_b = value;
    return FAC_OK;
  }
  if (k == "tail_only") {
    if (c->loaded) return set_err(c, FAC_ERR_ARG, "tail_only must be set before fac_load_weights");
    c->tail_only = value != 0;
    return FAC_OK;
  }
  if (k == "fuse_stem224") {
    c->fuse_stem224 = value != 0;
    return FAC_OK;
  }
  if (k == "stem_events") {
    c->stem_ev = value != 0;
    c->stem_ev_used = 0;
    return FAC_OK;
  }
  if (k == "nd_occ3") {  // convnd_igemm 3-per-CU tile for cout <= 64 up to this many K steps (default 4; 0 = off); process-wide
    if (value < 0) return set_err(c, FAC_ERR_ARG, "nd_occ3 must be >= 0");
    fac::set_nd_occ3(value);
    return FAC_OK;
  }
  if (k == "nd_pt_wide") {  // convnd_pt for cout % 128 != 0 from this many 256-row tiles (default 32; 0: off); process-wide
    if (value < 0) return set_err(c, FAC_ERR_ARG, "nd_pt_wide must be >= 0");
    fac::set_nd_pt_wide(value);
    return FAC_OK;
  }
  if (k == "pool_roll") {  // MaxPool3d(3,1,1) on 7-wide maps: 1 (default) maxpool3_roll, k >= 2 k frames per thread, 0 maxpool3_s1; process-wide
    if (value < 0) return set_err(c, FAC_ERR_ARG, "pool_roll must be >= 0");
    fac::set_pool_roll(value);
    return FAC_OK;
  }
  if (k == "pool3_g") {  // frames per maxpool3_pw unit on 7x7 maps: 0 default (2), 1, 2 or 4; process-wide
    if (value != 0 && value != 1 && value != 2 && value != 4) return set_err(c, FAC_ERR_ARG, "pool3_g must be 0, 1, 2 or 4");
    fac::set_pool3_g(value);
    return FAC_OK;
  }
  if (k == "tk_wreg") {  // 1 (default): S3D's cin-128 / 192 temporal convs with the weights in VGPRs; 0: in LDS; process-wide
    fac::set_tk_wreg(value != 0);
    return FAC_OK;
  }
  if (k == "pw_res") {  // 1 (default): ResNet's K = 128 / 256 conv3 + identity by pw_res and layer2's
                        // conv3 + strided downsample by pw_dual2; 2: pw_res only; 0: convnd_pt; process-wide
    if (value < 0 || value > 2) return set_err(c, FAC_ERR_ARG, "pw_res must be 0, 1 or 2");
    fac::set_pw_res((int)value);
    return FAC_OK;
  }
  if (k == "pool_lds14") {  // 1 (default): MaxPool3d(3,1,1) on 14x14 maps by maxpool3_lds14; 0: maxpool3_s1; process-wide
    fac::set_pool_lds14(value != 0);
    return FAC_OK;
  }
  if (k == "pool3_zg") {  // output frames per thread of maxpool3_s1 (0 = all, the default); process-wide
    if (value < 0) return set_err(c, FAC_ERR_ARG, "pool3_zg must be >= 0");
    fac::set_pool3_zg(value);
    return FAC_OK;
  }
  if (k == "pool_win") {  // 1 (default): max pools with a (1,3,3) / (3,3,3) / (2,2,2) window by pool_max_win; 0: pool_nd; process-wide
    fac::set_pool_win(value != 0);
    return FAC_OK;
  }
  if (k == "stem_nwg") {
    if (value < 0) return set_err(c, FAC_ERR_ARG, "stem_nwg must be >= 0");
    c->stem_nwg = value;
    return FAC_OK;
  }
  static const char* gemm_keys[6] = {"gemm_patch", "gemm_qkv", "gemm_out", "gemm_ff1", "gemm_ff2", "gemm_head"};
  for (int i = 0; i < 6; ++i)
    if (k == gemm_keys[i]) {
      if (value < -1 || value > 6) return set_err(c, FAC_ERR_ARG, "gemm variant must be -1..6");
      c->gemm_var[i] = value;
      return FAC_OK;
    }
  if (k == "gemm_small") {  // process-wide: tile variant of GEMMs with <= 64 rows (default 5; -1: the wide tiles)
    if (value < -1 || value > 6) return set_err(c, FAC_ERR_ARG, "gemm_small must be -1..6");
    fac::set_gemm_small(value < 0 ? 0 : 64, value < 0 ? 0 : value);
    return FAC_OK;
  }
  if (k == "ffn_ln_eps_exp") {
    if (value < 1 || value > 12) return set_err(c, FAC_ERR_ARG, "ffn_ln_eps_exp must be 1..12");
    c->ffn_ln_eps = (float)std::pow(10.0, -value);
    return FAC_OK;
  }
  if (k == "tail_priority") {
    if (c->tail_st) return set_err(c, FAC_ERR_ARG, "tail_priority must be set before the first pipelined forward");
    c->tail_priority = value != 0;
    return FAC_OK;
  }
  if (k == "proj_splits") {
    if (value != 1 && value != 2 && value != 4) return set_err(c, FAC_ERR_ARG, "proj_splits must be 1, 2 or 4");
    c->proj_splits = value;
    return FAC_OK;
  }
  return set_err(c, FAC_ERR_ARG, "unknown option " + k);
}

int fac_forward_features(fac_ctx* c, const void* d_feat, int B, const int32_t* d_pos, float* d_hidden,
                         float* d_logits, float* d_probs, void* stream) {
  if (!c) return FAC_ERR_ARG;
  if (!c->loaded) return set_err(c, FAC_ERR_NOT_LOADED, "forward before fac_load_weights");
  if (!d_feat || !d_pos || B <= 0 || (!d_hidden && !d_logits))
    return set_err(c, FAC_ERR_ARG, "bad fac_forward_features arguments");
  if (B > 32 * 1024) return set_err(c, FAC_ERR_SHAPE, "batch too large");
  if (int e = take_device_error(c)) return e;
  DevGuard g(c->device);
  int rc = ensure_ws(c, B);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_TRY(c, hipStreamIsCapturing(st, &cs));
  if (cs != hipStreamCaptureStatusNone) {
    for (int i = 0; i < 2; ++i)
      if (c->tail_pending[i]) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_tail[i], 0));
    return tail_impl(c, (const uint16_t*)d_feat, B, d_pos, d_logits, d_probs, st, nullptr, d_hidden);
  }
  rc = order_on(c, st);  // the shared encoder buffers: after the context's previous forward on any stream
  if (rc) return rc;
  rc = tail_impl(c, (const uint16_t*)d_feat, B, d_pos, d_logits, d_probs, st, nullptr, d_hidden);
  if (rc) return rc;
  return mark_done(c, st);
}

int fac_forward_nchw_f32(fac_ctx* c, const float* d_in, int B, const int32_t* d_pos, float* d_logits, float* d_probs,
                         void* stream) {
  return forward_entry(c, d_in, false, B, d_pos, d_logits, d_probs, stream);
}

int fac_forward_nhwc_u8(fac_ctx* c, const uint8_t* d_in, int B, const int32_t* d_pos, float* d_logits, float* d_probs,
                        void* stream) {
  return forward_entry(c, d_in, true, B, d_pos, d_logits, d_probs, stream);
}

int fac_forward_nhwc_u8_pipelined(fac_ctx* c, const uint8_t* d_in, int B, const int32_t* d_pos, float* d_logits,
                                  float* d_probs, float* d_score, void* stream) {
  if (!c) return FAC_ERR_ARG;
  if (!c->loaded) return set_err(c, FAC_ERR_NOT_LOADED, "forward before fac_load_weights");
  if (!d_in || !d_pos || !d_logits || B <= 0) return set_err(c, FAC_ERR_ARG, "bad pipelined forward arguments");
  DevGuard g(c->device);
  if (!c->tail_st) {
    // the encoder's short, latency-bound kernels get the higher priority, so
    // the dispatcher slots their workgroups in as the conv stack's retire
    int lo = 0, hi = 0;
    HIP_TRY(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(c, hipStreamCreateWithPriority(&c->tail_st, hipStreamNonBlocking, c->tail_priority ? hi : lo));
    for (int i = 0; i < 2; ++i) {
      HIP_TRY(c, hipEventCreateWithFlags(&c->ev_conv[i], hipEventDisableTiming));
      HIP_TRY(c, hipEventCreateWithFlags(&c->ev_tail[i], hipEventDisableTiming));
    }
  }
  if (B > c->cap_B && (c->tail_pending[0] || c->tail_pending[1]))
    HIP_TRY(c, hipStreamSynchronize(c->tail_st));  // the workspace is about to be reallocated
  int rc = ensure_ws(c, B);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const int k = c->pipe_k & 1;
  uint16_t* stem = k ? c->stem_out2 : c->stem_out;
  // stem buffer k was last read by the tail of batch k-2
  if (c->tail_pending[k]) HIP_TRY(c, hipStreamWaitEvent(st, c->ev_tail[k], 0));
  rc = forward_impl(c, d_in, true, B, nullptr, nullptr, nullptr, stream, nullptr, -1, nullptr, nullptr, stem, true);
  if (rc) return rc;
  HIP_TRY(c, hipEventRecord(c->ev_conv[k], st));
  HIP_TRY(c, hipStreamWaitEvent(c->tail_st, c->ev_conv[k], 0));
  rc = tail_impl(c, stem, B, d_pos, d_logits, d_probs, c->tail_st, nullptr, nullptr, true);
  if (rc) return rc;
  if (d_score) HIP_TRY(c, fac::launch_video_score(d_logits, B, d_score, c->tail_st));
  HIP_TRY(c, hipEventRecord(c->ev_tail[k], c->tail_st));
  c->tail_pending[k] = true;
  c->pipe_k++;
  return FAC_OK;
}

int fac_pipeline_join(fac_ctx* c, int keep, void* stream) {
  if (!c || keep < 0) return FAC_ERR_ARG;
  if (!c->tail_st) return FAC_OK;
  DevGuard g(c->device);
  // the batches enqueued, oldest first: pipe_k-2, pipe_k-1 (slots (pipe_k-2)&1, (pipe_k-1)&1)
  for (int age = 2; age > keep; --age) {
    const int k = (c->pipe_k - age) & 1;
    if (c->pipe_k - age >= 0 && c->tail_pending[k])
      HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_tail[k], 0));
  }
  return FAC_OK;
}

int fac_debug_gemm(fac_ctx* c, int epi, const uint16_t* d_a, const uint16_t* d_w, const float* d_bias, void* d_out,
                   int M, int N, int K, int splits, int variant, void* stream) {
  if (!c || !d_a || !d_w || !d_out) return set_err(c, FAC_ERR_ARG, "bad debug_gemm arguments");
  const hipError_t e = fac::launch_gemm(c->dtype, epi, d_a, K, d_w, K, d_bias, d_out, N, M, N, K, splits,
                                   (hipStream_t)stream, variant);
  if (e != hipSuccess) return set_err(c, e == hipErrorInvalidValue ? FAC_ERR_ARG : FAC_ERR_HIP,
                                      std::string("debug_gemm: ") + hipGetErrorString(e));
  return FAC_OK;
}

int fac_debug_features_u8(fac_ctx* c, const uint8_t* d_in, int B, int layer, uint16_t* d_out, void* stream) {
  if (!c || !d_out || layer < 0 || layer > 16) return set_err(c, FAC_ERR_ARG, "bad debug_features arguments");
  return forward_impl(c, d_in, true, B, nullptr, nullptr, nullptr, stream, nullptr, layer, d_out);
}

int fac_debug_conv(fac_ctx* c, int layer, const uint16_t* d_in, int B, uint16_t* d_out, void* stream) {
  if (!c || !d_in || !d_out || B <= 0 || layer < 1 || layer > 16) return set_err(c, FAC_ERR_ARG, "bad debug_conv arguments");
  if (!c->loaded) return set_err(c, FAC_ERR_NOT_LOADED, "debug_conv before fac_load_weights");
  DevGuard g(c->device);
  const ConvLayer& L = c->conv[layer - 1];
  HIP_TRY(c, run_conv(c, L, d_in, d_out, B, (hipStream_t)stream));
  return FAC_OK;
}

int fac_debug_tail(fac_ctx* c, const uint16_t* d_stem, int B, const int32_t* d_pos, float* d_logits, void* stream) {
  if (!d_stem) return set_err(c, FAC_ERR_ARG, "bad debug_tail arguments");
  return forward_impl(c, nullptr, true, B, d_pos, d_logits, nullptr, stream, nullptr, -1, nullptr, d_stem);
}

int fac_profile_forward_u8(fac_ctx* c, const uint8_t* d_in, int B, const int32_t* d_pos, float* d_logits,
                           float* stage_ms, int n_stages, void* stream) {
  if (!c || !stage_ms || n_stages < FAC_PROFILE_STAGES) return set_err(c, FAC_ERR_ARG, "bad profile arguments");
  DevGuard g(c->device);
  Prof p;
  int rc = forward_impl(c, d_in, true, B, d_pos, d_logits, nullptr, stream, &p);
  for (int i = 0; i < FAC_PROFILE_STAGES; ++i) stage_ms[i] = 0.f;
  if (rc == FAC_OK && !p.ev.empty()) {
    HIP_TRY(c, hipEventSynchronize(p.ev.back()));
    for (size_t i = 1; i < p.ev.size(); ++i) {
      if (p.stage[i] < 0 || p.stage[i] >= FAC_PROFILE_STAGES) continue;
      float ms = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&ms, p.ev[i - 1], p.ev[i]));
      stage_ms[p.stage[i]] += ms;
    }
  }
  for (hipEvent_t e : p.ev) (void)hipEventDestroy(e);
  return rc;
}

int fac_stem_event_ms(fac_ctx* c, float* avg_ms, int* n_launches) {
  if (!c || !avg_ms || !n_launches) return FAC_ERR_ARG;
  DevGuard g(c->device);
  *avg_ms = 0.f;
  *n_launches = (int)(c->stem_ev_used / 2);
  if (!*n_launches) return FAC_OK;
  HIP_TRY(c, hipEventSynchronize(c->stem_evs[c->stem_ev_used - 1]));
  double sum = 0.0;
  for (size_t i = 0; i < c->stem_ev_used; i += 2) {
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->stem_evs[i], c->stem_evs[i + 1]));
    sum += ms;
  }
  *avg_ms = (float)(sum / *n_launches);
  c->stem_ev_used = 0;
  return FAC_OK;
}

int fac_check_device_errors(fac_ctx* c, int* flags) {
  if (!c || !flags) return FAC_ERR_ARG;
  *flags = 0;
  if (!c->err_host) return FAC_OK;
  DevGuard g(c->device);
  HIP_TRY(c, hipDeviceSynchronize());
  *flags = *(volatile int*)c->err_host;
  *(volatile int*)c->err_host = 0;
  return FAC_OK;
}

int fac_video_score(const float* d_logits, int n, float* d_score, void* stream) {
  if (!d_score || n < 0 || (n > 0 && !d_logits)) return FAC_ERR_ARG;
  return fac::launch_video_score(d_logits, n, d_score, (hipStream_t)stream) == hipSuccess ? FAC_OK : FAC_ERR_HIP;
}

int fac_video_score_seg(const float* d_logits, const int* d_seg, int nv, float* d_scores, void* stream) {
  if (nv < 0 || (nv > 0 && (!d_logits || !d_seg || !d_scores))) return FAC_ERR_ARG;
  if (nv == 0) return FAC_OK;
  return fac::launch_video_score_seg(d_logits, d_seg, nv, d_scores, (hipStream_t)stream) == hipSuccess ? FAC_OK
                                                                                                   : FAC_ERR_HIP;
}

const char* fac_last_error(fac_ctx* c) { return c ? c->err.c_str() : "null context"; }

void fac_destroy(fac_ctx* c) {
  if (!c) return;
  {
    DevGuard g(c->device);
    (void)hipDeviceSynchronize();
    if (c->tail_st) {
      (void)hipStreamDestroy(c->tail_st);
      for (int i = 0; i < 2; ++i) {
        (void)hipEventDestroy(c->ev_conv[i]);
        (void)hipEventDestroy(c->ev_tail[i]);
      }
    }
    for (hipEvent_t e : c->stem_evs) (void)hipEventDestroy(e);
    if (c->ev_stack) (void)hipEventDestroy(c->ev_stack);
    drop_graphs(c);
    if (c->cap_st) (void)hipStreamDestroy(c->cap_st);
    for (void* p : c->g_in)
      if (p) (void)hipFree(p);
    if (c->g_pidx) (void)hipFree(c->g_pidx);
    if (c->g_out) (void)hipFree(c->g_out);
    for (void* p : c->weights) (void)hipFree(p);
    if (c->ws) (void)hipFree(c->ws);
    if (c->err_host) (void)hipHostFree(c->err_host);
  }
  delete c;
}

int fac_crop_resize_u8(const uint8_t* d_frames, int n_frames, int H, int W, const int32_t* d_boxes, int n_boxes,
                       uint8_t* d_crops, void* stream) {
  if (!d_frames || !d_boxes || !d_crops || n_frames <= 0 || H <= 0 || W <= 0 || n_boxes < 0) return FAC_ERR_ARG;
  if ((long long)n_frames * H * W * 3 >= (1ll << 40)) return FAC_ERR_SHAPE;
  return fac::launch_crop_resize(d_frames, n_frames, H, W, d_boxes, n_boxes, d_crops, (hipStream_t)stream) ==
                 hipSuccess
             ? FAC_OK
             : FAC_ERR_HIP;
}

const char* fac_version(void) { return "fac_cvit 0.1.0 (gfx950, MFMA 16x16x32 bf16/f16)"; }

}  // extern "C"
