// Image preprocessing of the eval loaders: the reference's get_transform
// (visreps/dataloaders/obj_cls.py:27-45)
//   Resize(resize, BILINEAR) -> CenterCrop(crop) -> ToTensor -> Normalize(mean, std)
// on PIL images. torchvision hands a PIL image to Pillow's Image.resize, so the arithmetic
// to match is Pillow's ImagingResample (libImaging/Resample.c, Pillow 12):
//   * per output index a window [xmin, xmin + xmax) of input pixels with filter weights
//     f((x + xmin - center + 0.5) / filterscale) (f: Pillow's bilinear tent, or its bicubic
//     kernel with a = -0.5 for the CLIP / timm loaders), center = (xx + 0.5) * scale,
//     filterscale = max(scale, 1) (the support widens when downscaling: antialiasing),
//     normalised to sum 1 in double, then rounded to 22-bit fixed point;
//   * a horizontal pass into a uint8 intermediate, then a vertical pass, each output
//     (2^21 + sum in[i] k[i]) >> 22 clamped to [0, 255];
// and torchvision's resize size (shorter side -> resize, longer side int(resize * long /
// short)), center-crop offsets int(round((size - crop) / 2)) (half to even), ToTensor's
// v / 255 and Normalize's (x - mean) / std, each one fp32 operation.
//
// Three kernels per batch of same-size images (B x H x W x 3 uint8, device memory):
//  k_tf_coeffs  the Pillow coefficient tables for the crop's columns and rows, in fp64 on
//               the device with contraction off (the x86 build of Pillow computes them
//               with separate IEEE multiplies and adds; fp64 +,-,*,/ and ceil are exact-
//               rounded on CDNA4, so the tables are bit-identical)
//  k_tf_horiz   the intermediate rows the crop needs, crop columns only (uint8)
//  k_tf_vert    vertical pass + /255 + normalise -> out (B x 3 x crop x crop fp32)
// Everything is integer or exact-rounded fp32, so the output equals torchvision on PIL
// bit for bit (tests/test_transform.py checks it against Pillow itself).
#include "internal.h"

#include <cmath>

namespace vr {

constexpr int TF_PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2

struct TfGeom {
  int filter;          // 0 bilinear (support 1), 1 bicubic (support 2, a = -0.5)
  int64_t H, W;        // input
  int64_t nh, nw;      // resized
  int64_t crop, top, left;
  int kh, kv;          // coefficients per output column / row (ksize)
  int64_t r0, nrows;   // intermediate rows [r0, r0 + nrows) needed by the crop's rows
};

static int64_t round_half_even(double v) { return (int64_t)std::nearbyint(v); }

static double filter_support(int filter) { return filter == 1 ? 2.0 : 1.0; }

static int ksize_of(int64_t in, int64_t out, int filter) {
  double fs = (double)in / (double)out;
  if (fs < 1.0) fs = 1.0;
  return (int)std::ceil(filter_support(filter) * fs) * 2 + 1;
}

// torchvision _compute_resized_output_size (size = [resize], no max_size)
static TfGeom tf_geom(int64_t H, int64_t W, int64_t resize, int64_t crop, int filter) {
  TfGeom g;
  g.filter = filter;
  g.H = H;
  g.W = W;
  const int64_t s = W <= H ? W : H, l = W <= H ? H : W;
  const int64_t ns = resize, nl = (int64_t)((double)resize * (double)l / (double)s);
  g.nw = W <= H ? ns : nl;
  g.nh = W <= H ? nl : ns;
  g.crop = crop;
  g.top = round_half_even((double)(g.nh - crop) / 2.0);
  g.left = round_half_even((double)(g.nw - crop) / 2.0);
  g.kh = ksize_of(W, g.nw, filter);
  g.kv = ksize_of(H, g.nh, filter);
  g.r0 = 0;
  g.nrows = 0;
  return g;
}

struct TfWs {
  int32_t* kh;  // [crop][kh] horizontal coefficients of the crop's columns
  int32_t* bh;  // [crop][2]  (xmin, xmax)
  int32_t* kv;  // [crop][kv]
  int32_t* bv;  // [crop][2]
  uint8_t* tmp; // [B][nrows][crop][3]
};

static TfWs tf_layout(void* base, int64_t B, const TfGeom& g, int64_t max_rows, size_t* bytes) {
  Carver c(base);
  TfWs w;
  w.kh = c.take<int32_t>((size_t)g.crop * g.kh);
  w.bh = c.take<int32_t>((size_t)g.crop * 2);
  w.kv = c.take<int32_t>((size_t)g.crop * g.kv);
  w.bv = c.take<int32_t>((size_t)g.crop * 2);
  w.tmp = c.take<uint8_t>((size_t)B * max_rows * g.crop * 3);
  if (bytes) *bytes = c.bytes();
  return w;
}

// Pillow's filters (Resample.c bilinear_filter, bicubic_filter with a = -0.5)
__device__ inline double tf_filter(int filter, double x) {
#pragma clang fp contract(off)
  if (x < 0.0) x = -x;
  if (filter == 1) {
    const double a = -0.5;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
  }
  return x < 1.0 ? 1.0 - x : 0.0;
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc for output index xx of an in -> out
// resize (box [0, in)). One thread per output index.
__device__ void tf_coeff_one(int filter, int64_t in, int64_t out, int64_t xx, int ksize, int32_t* k,
                             int32_t* bounds) {
#pragma clang fp contract(off)
  const double scale = (double)(float)((float)in - 0.0f) / (double)out;
  double filterscale = scale;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = (filter == 1 ? 2.0 : 1.0) * filterscale;
  const double center = 0.0 + ((double)xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in) xmax = (int)in;
  xmax -= xmin;
  double w[64];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    const double v = tf_filter(filter, ((double)(x + xmin) - center + 0.5) * ss);
    w[x] = v;
    ww += v;
  }
  for (int x = 0; x < ksize; ++x) {
    double v = x < xmax ? w[x] : 0.0;
    if (x < xmax && ww != 0.0) v /= ww;
    const double f = v * (double)(1 << TF_PREC);
    k[x] = v < 0 ? (int32_t)(-0.5 + f) : (int32_t)(0.5 + f);
  }
  bounds[0] = xmin;
  bounds[1] = xmax;
}

__global__ void k_tf_coeffs(TfGeom g, TfWs w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < g.crop) tf_coeff_one(g.filter, g.W, g.nw, g.left + i, g.kh, w.kh + i * g.kh, w.bh + 2 * i);
  else if (i < 2 * g.crop) {
    const int64_t j = i - g.crop;
    tf_coeff_one(g.filter, g.H, g.nh, g.top + j, g.kv, w.kv + j * g.kv, w.bv + 2 * j);
  }
}

__device__ inline uint8_t tf_clip8(int32_t v) {
  const int32_t s = v >> TF_PREC;  // arithmetic shift, as Pillow's clip8 table index
  return (uint8_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}

// tmp[b][r][x][c] = horizontal pass of input row r0 + r at crop column x
__global__ __launch_bounds__(256) void k_tf_horiz(const uint8_t* __restrict__ src, int64_t B, TfGeom g,
                                                  TfWs w) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = blockIdx.y, b = blockIdx.z;
  if (x >= g.crop || b >= B) return;
  const int32_t xmin = w.bh[2 * x], xmax = w.bh[2 * x + 1];
  const int32_t* k = w.kh + x * g.kh;
  const uint8_t* row = src + ((size_t)b * g.H + (size_t)(g.r0 + r)) * (size_t)g.W * 3;
  int32_t s0 = 1 << (TF_PREC - 1), s1 = s0, s2 = s0;
  for (int32_t i = 0; i < xmax; ++i) {
    const uint8_t* p = row + (size_t)(xmin + i) * 3;
    s0 += (int32_t)p[0] * k[i];
    s1 += (int32_t)p[1] * k[i];
    s2 += (int32_t)p[2] * k[i];
  }
  uint8_t* o = w.tmp + (((size_t)b * g.nrows + r) * g.crop + x) * 3;
  o[0] = tf_clip8(s0);
  o[1] = tf_clip8(s1);
  o[2] = tf_clip8(s2);
}

struct TfNorm {
  float mean[3], std[3];
};

__global__ __launch_bounds__(256) void k_tf_vert(int64_t B, TfGeom g, TfWs w, TfNorm nm,
                                                 float* __restrict__ out) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t y = blockIdx.y, b = blockIdx.z;
  if (x >= g.crop || b >= B) return;
  const int32_t ymin = w.bv[2 * y] - (int32_t)g.r0, ymax = w.bv[2 * y + 1];
  const int32_t* k = w.kv + y * g.kv;
  int32_t s[3] = {1 << (TF_PREC - 1), 1 << (TF_PREC - 1), 1 << (TF_PREC - 1)};
  for (int32_t i = 0; i < ymax; ++i) {
    const uint8_t* p = w.tmp + (((size_t)b * g.nrows + (size_t)(ymin + i)) * g.crop + x) * 3;
    s[0] += (int32_t)p[0] * k[i];
    s[1] += (int32_t)p[1] * k[i];
    s[2] += (int32_t)p[2] * k[i];
  }
  const size_t plane = (size_t)g.crop * g.crop;
  float* o = out + (size_t)b * 3 * plane + (size_t)y * g.crop + x;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = __fdiv_rn((float)tf_clip8(s[c]), 255.0f);  // ToTensor
    o[c * plane] = __fdiv_rn(__fsub_rn(v, nm.mean[c]), nm.std[c]);  // Normalize
  }
}

// rows of the input the crop's output rows read: Pillow's bounds, evaluated on the host
// with the same double arithmetic (only to size the intermediate; the kernel tables are
// the ones used)
static void tf_rows(TfGeom& g) {
  const double scale = (double)g.H / (double)g.nh;
  const double fs = (scale < 1.0 ? 1.0 : scale) * filter_support(g.filter);
  auto lo = [&](int64_t yy) {
    const double c = ((double)yy + 0.5) * scale;
    int64_t m = (int64_t)(c - fs + 0.5);
    return m < 0 ? (int64_t)0 : m;
  };
  auto hi = [&](int64_t yy) {
    const double c = ((double)yy + 0.5) * scale;
    int64_t m = (int64_t)(c + fs + 0.5);
    return m > g.H ? g.H : m;
  };
  // one row of slack each side covers any last-bit difference of the host estimate
  g.r0 = std::max<int64_t>(0, lo(g.top) - 1);
  const int64_t r1 = std::min<int64_t>(g.H, hi(g.top + g.crop - 1) + 1);
  g.nrows = r1 - g.r0;
}

}  // namespace vr

using namespace vr;

extern "C" {

size_t vr_transform_workspace(int64_t B, int64_t H, int64_t W, int64_t resize, int64_t crop,
                              int filter) {
  if (B <= 0 || H <= 0 || W <= 0 || resize <= 0 || crop <= 0 || filter < 0 || filter > 1) return 0;
  TfGeom g = tf_geom(H, W, resize, crop, filter);
  tf_rows(g);
  size_t bytes = 0;
  tf_layout(nullptr, B, g, g.nrows, &bytes);
  return bytes;
}

int vr_transform_u8(const uint8_t* src, int64_t B, int64_t H, int64_t W, int64_t resize,
                    int64_t crop, int filter, const float* mean, const float* std, float* out,
                    void* ws, size_t ws_bytes, void* stream) {
  VR_REQUIRE(filter == 0 || filter == 1, "vr_transform_u8: filter %d (0 bilinear, 1 bicubic)", filter);
  VR_REQUIRE(B >= 0 && H > 0 && W > 0 && resize > 0 && crop > 0,
             "vr_transform_u8: bad shape B=%lld H=%lld W=%lld resize=%lld crop=%lld", (long long)B,
             (long long)H, (long long)W, (long long)resize, (long long)crop);
  if (B == 0) return VR_OK;
  VR_REQUIRE(src && out && mean && std && ws, "vr_transform_u8: null pointer");
  TfGeom g = tf_geom(H, W, resize, crop, filter);
  VR_REQUIRE(crop <= g.nh && crop <= g.nw,
             "vr_transform_u8: crop %lld larger than the resized image %lldx%lld (torchvision pads)",
             (long long)crop, (long long)g.nh, (long long)g.nw);
  VR_REQUIRE(g.kh <= 64 && g.kv <= 64, "vr_transform_u8: downscale factor too large (W=%lld H=%lld)",
             (long long)W, (long long)H);
  tf_rows(g);
  size_t need = 0;
  const TfWs w = tf_layout(ws, B, g, g.nrows, &need);
  VR_REQUIRE(ws_bytes >= need, "vr_transform_u8: workspace %zu < %zu", ws_bytes, need);
  VR_REQUIRE(B <= 65535 && g.nrows <= 65535, "vr_transform_u8: batch too large");
  hipStream_t st = as_stream(stream);
  TfNorm nm;
  for (int c = 0; c < 3; ++c) {
    nm.mean[c] = mean[c];
    nm.std[c] = std[c];
  }
  k_tf_coeffs<<<(unsigned)((2 * crop + 127) / 128), 128, 0, st>>>(g, w);
  VR_CHECK_LAUNCH();
  const unsigned gx = (unsigned)((crop + 255) / 256);
  k_tf_horiz<<<dim3(gx, (unsigned)g.nrows, (unsigned)B), 256, 0, st>>>(src, B, g, w);
  VR_CHECK_LAUNCH();
  k_tf_vert<<<dim3(gx, (unsigned)crop, (unsigned)B), 256, 0, st>>>(B, g, w, nm, out);
  VR_CHECK_LAUNCH();
  return VR_OK;
}

}  // extern "C"
