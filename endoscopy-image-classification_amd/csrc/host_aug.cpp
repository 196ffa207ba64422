// Host-side input path for real-data runs: the reference's torchvision /
// PIL transforms for the SSL trainers, as native C++ over RGB uint8 images, with a multi-threaded
// batch builder that writes the planar uint8 [n, 3, S, S] batches the device path consumes
// (es_patch_im2col_u8 fuses ToTensor + Normalize into the patch gather, so the host never makes fp32).
//
// Reference behaviour restated (code/randaugment.py, code/dataset.py:24-56,185-207), on the PIL
// algorithms those transforms call; every op is pinned bit-exact to PIL by tests/test_host_aug.py:
//   ImageOps.autocontrast / equalize / posterize / solarize            (per-band LUTs)
//   ImageEnhance.Brightness / Color / Contrast / Sharpness             (Image.blend with a degenerate)
//   Image.rotate / Image.transform(AFFINE), NEAREST                     (16.16 fixed-point walk, or the
//                                                                        scale-only table for translations)
//   Image.resize(BILINEAR)                                              (two-pass separable, 22-bit coefficients)
//   ImageDraw.rectangle (Cutout: inclusive corners), flips, crops, reflect padding (numpy 'reflect')
//
// Images: HWC, 3 bytes per pixel, rows contiguous (w * 3 bytes).  Randomness: the reference draws from
// Python's `random`, numpy and torch generators; here every image owns a counter-based stream keyed on
// (batch seed, image index), so a batch is identical for any thread count.  The DISTRIBUTIONS are the
// reference's (op choice with replacement, magnitude randint(1, m), apply / sign / flip probability 0.5,
// crop offsets uniform over the valid range, Cutout centre uniform over the image).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

using u8 = uint8_t;

// ---- per-image random stream (splitmix64 over a counter) --------------------------------------
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0, 1)
  int randint(int lo, int hi_excl) {  // [lo, hi)
    const uint64_t span = (uint64_t)(hi_excl - lo);
    return lo + (int)(next() % span);
  }
};

uint64_t image_seed(uint64_t seed, uint64_t index, uint64_t stream) {
  Rng r(seed ^ (index * 0xD1B54A32D192ED03ull) ^ (stream * 0x8CB92BA72F3D8DD7ull));
  r.next();
  return r.next();
}

// Pixel buffers come from a process-wide free list: a 150-KB image is past glibc's mmap threshold, and
// a fresh mmap per temporary costs a munmap (a TLB shootdown across the worker threads) plus first-touch
// page faults on every use; batch threads are short-lived, so the list is shared, not thread-local.
std::mutex g_buf_mu;
std::vector<std::vector<u8>> g_bufs;
constexpr size_t MAX_CACHED_BUFS = 96;

std::vector<u8> take_buf(size_t n) {
  {
    std::lock_guard<std::mutex> lk(g_buf_mu);
    size_t best = g_bufs.size();
    for (size_t i = 0; i < g_bufs.size(); ++i)  // smallest buffer that fits
      if (g_bufs[i].capacity() >= n && (best == g_bufs.size() || g_bufs[i].capacity() < g_bufs[best].capacity()))
        best = i;
    if (best < g_bufs.size()) {
      std::vector<u8> v = std::move(g_bufs[best]);
      g_bufs[best] = std::move(g_bufs.back());
      g_bufs.pop_back();
      v.resize(n);  // contents unspecified: every producer writes all of it (Img::zeros where it must be 0)
      return v;
    }
  }
  std::vector<u8> v;
  v.reserve(n);
  v.resize(n);
  return v;
}

constexpr size_t MAX_CACHED_BYTES = (size_t)4 << 20;  // larger temporaries (huge sources) go back to malloc

void give_buf(std::vector<u8>&& v) {
  if (!v.capacity() || v.capacity() > MAX_CACHED_BYTES) return;
  std::lock_guard<std::mutex> lk(g_buf_mu);
  if (g_bufs.size() < MAX_CACHED_BUFS) g_bufs.push_back(std::move(v));
}

struct Img {
  int w = 0, h = 0;
  std::vector<u8> px;
  Img() = default;
  Img(int w_, int h_) : w(w_), h(h_), px(take_buf((size_t)w_ * h_ * 3)) {}
  Img(const Img& o) : w(o.w), h(o.h), px(take_buf(o.px.size())) { std::memcpy(px.data(), o.px.data(), px.size()); }
  Img(Img&& o) noexcept : w(o.w), h(o.h), px(std::move(o.px)) {}
  Img& operator=(const Img& o) {
    if (this != &o) {
      if (px.capacity() < o.px.size()) { give_buf(std::move(px)); px = take_buf(o.px.size()); }
      px.resize(o.px.size());
      std::memcpy(px.data(), o.px.data(), px.size());
      w = o.w;
      h = o.h;
    }
    return *this;
  }
  Img& operator=(Img&& o) noexcept {
    if (this != &o) {
      give_buf(std::move(px));
      px = std::move(o.px);
      w = o.w;
      h = o.h;
    }
    return *this;
  }
  ~Img() { give_buf(std::move(px)); }
  static Img zeros(int w_, int h_) {
    Img z(w_, h_);
    std::memset(z.px.data(), 0, z.px.size());
    return z;
  }
  u8* row(int y) { return px.data() + (size_t)y * w * 3; }
  const u8* row(int y) const { return px.data() + (size_t)y * w * 3; }
};

struct View {  // a caller's image, read in place
  const u8* p;
  int w, h;
  const u8* row(int y) const { return p + (size_t)y * w * 3; }
};

Img from_ptr(const u8* p, int w, int h) {
  Img im(w, h);
  std::memcpy(im.px.data(), p, im.px.size());
  return im;
}

// ---- LUT ops (PIL/ImageOps.py) -----------------------------------------------------------------
void apply_lut3(Img& im, const int lut[3][256]) {
  u8* p = im.px.data();
  const size_t n = (size_t)im.w * im.h;
  for (size_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) p[i * 3 + c] = (u8)lut[c][p[i * 3 + c]];
}

void histogram3(const Img& im, long hist[3][256]) {
  std::memset(hist, 0, sizeof(long) * 3 * 256);
  const u8* p = im.px.data();
  const size_t n = (size_t)im.w * im.h;
  for (size_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) ++hist[c][p[i * 3 + c]];
}

void autocontrast(Img& im) {  // ImageOps.autocontrast(img), cutoff 0
  long hist[3][256];
  histogram3(im, hist);
  int lut[3][256];
  for (int c = 0; c < 3; ++c) {
    int lo = 0, hi = 255;
    while (lo < 255 && !hist[c][lo]) ++lo;
    while (hi > 0 && !hist[c][hi]) --hi;
    if (hi <= lo) {
      for (int i = 0; i < 256; ++i) lut[c][i] = i;
    } else {
      const double scale = 255.0 / (hi - lo), offset = -lo * scale;
      for (int i = 0; i < 256; ++i) {
        int v = (int)(i * scale + offset);  // Python int(): truncation toward zero
        lut[c][i] = v < 0 ? 0 : (v > 255 ? 255 : v);
      }
    }
  }
  apply_lut3(im, lut);
}

void equalize(Img& im) {  // ImageOps.equalize(img)
  long hist[3][256];
  histogram3(im, hist);
  int lut[3][256];
  for (int c = 0; c < 3; ++c) {
    long total = 0, last = 0;
    int nz = 0;
    for (int i = 0; i < 256; ++i)
      if (hist[c][i]) { total += hist[c][i]; last = hist[c][i]; ++nz; }
    const long step = nz <= 1 ? 0 : (total - last) / 255;
    if (!step) {
      for (int i = 0; i < 256; ++i) lut[c][i] = i;
    } else {
      long n = step / 2;
      for (int i = 0; i < 256; ++i) {
        const long v = n / step;
        lut[c][i] = (int)v;  // PIL point() clips LUT entries to [0, 255]
        if (lut[c][i] > 255) lut[c][i] = 255;
        n += hist[c][i];
      }
    }
  }
  apply_lut3(im, lut);
}

void lut_same(Img& im, const int l[256]) {
  int lut[3][256];
  for (int c = 0; c < 3; ++c) std::memcpy(lut[c], l, sizeof(int) * 256);
  apply_lut3(im, lut);
}

void posterize(Img& im, int bits) {
  const int mask = ~((1 << (8 - bits)) - 1);
  int l[256];
  for (int i = 0; i < 256; ++i) l[i] = i & mask & 255;
  lut_same(im, l);
}

void solarize(Img& im, int threshold) {
  int l[256];
  for (int i = 0; i < 256; ++i) l[i] = i < threshold ? i : 255 - i;
  lut_same(im, l);
}

// ---- Image.blend and the ImageEnhance degenerates ---------------------------------------------
// out = deg + alpha * (img - deg) in float, truncated (clipped when alpha is outside [0, 1]);
// alpha == 0 / 1 copy an input (Pillow's ImagingBlend).
void blend_into(Img& im, const Img& deg, float alpha) {
  if (alpha == 0.0f) { im.px = deg.px; return; }
  if (alpha == 1.0f) return;
  u8* p = im.px.data();
  const u8* d = deg.px.data();
  const size_t n = im.px.size();
  if (alpha >= 0.0f && alpha <= 1.0f) {
    for (size_t i = 0; i < n; ++i) p[i] = (u8)(int)((float)(int)d[i] + alpha * (float)((int)p[i] - (int)d[i]));
  } else {
    for (size_t i = 0; i < n; ++i) {
      const float t = (float)(int)d[i] + alpha * (float)((int)p[i] - (int)d[i]);
      p[i] = t <= 0.0f ? 0 : (t >= 255.0f ? 255 : (u8)(int)t);
    }
  }
}

// blend against a constant degenerate (Brightness: 0, Contrast: the mean gray), same arithmetic
void blend_const(Img& im, int dv, float alpha) {
  if (alpha == 0.0f) { std::memset(im.px.data(), dv, im.px.size()); return; }
  if (alpha == 1.0f) return;
  u8* p = im.px.data();
  const size_t n = im.px.size();
  const float d = (float)dv;
  if (alpha >= 0.0f && alpha <= 1.0f) {
    for (size_t i = 0; i < n; ++i) p[i] = (u8)(int)(d + alpha * (float)((int)p[i] - dv));
  } else {
    for (size_t i = 0; i < n; ++i) {
      const float t = d + alpha * (float)((int)p[i] - dv);
      p[i] = t <= 0.0f ? 0 : (t >= 255.0f ? 255 : (u8)(int)t);
    }
  }
}

inline int luma(const u8* q) { return (q[0] * 19595 + q[1] * 38470 + q[2] * 7471 + 0x8000) >> 16; }  // convert("L")

void brightness(Img& im, float f) { blend_const(im, 0, f); }  // degenerate: black

void color(Img& im, float f) {
  Img deg(im.w, im.h);
  const size_t n = (size_t)im.w * im.h;
  for (size_t i = 0; i < n; ++i) {
    const u8 l = (u8)luma(&im.px[i * 3]);
    deg.px[i * 3] = deg.px[i * 3 + 1] = deg.px[i * 3 + 2] = l;
  }
  blend_into(im, deg, f);
}

void contrast(Img& im, float f) {
  // ImageStat.Stat(img.convert("L")).mean[0]: sum of i * hist[i] in double, over the pixel count
  long hist[256] = {0};
  const size_t n = (size_t)im.w * im.h;
  for (size_t i = 0; i < n; ++i) ++hist[luma(&im.px[i * 3])];
  double sum = 0.0;
  for (int i = 0; i < 256; ++i) sum += (double)i * (double)hist[i];
  const int mean = (int)(sum / (double)n + 0.5);
  blend_const(im, mean, f);
}

void sharpness(Img& im, float f) {
  // degenerate = img.filter(ImageFilter.SMOOTH): 3x3 kernel (1 1 1 / 1 5 1 / 1 1 1) / 13 in fp32,
  // rounded to nearest; the border rows and columns copied
  Img deg = im;
  const float k1 = 1.0f / 13.0f, k5 = 5.0f / 13.0f;
  for (int y = 1; y < im.h - 1; ++y) {
    const u8* r0 = im.row(y - 1);
    const u8* r1 = im.row(y);
    const u8* r2 = im.row(y + 1);
    u8* o = deg.row(y);
    for (int x = 1; x < im.w - 1; ++x)
      for (int c = 0; c < 3; ++c) {
        const int i = x * 3 + c;
        float ss = 0.0f;
        ss += (float)r2[i - 3] * k1 + (float)r2[i] * k1 + (float)r2[i + 3] * k1;
        ss += (float)r1[i - 3] * k1 + (float)r1[i] * k5 + (float)r1[i + 3] * k1;
        ss += (float)r0[i - 3] * k1 + (float)r0[i] * k1 + (float)r0[i + 3] * k1;
        o[i] = ss <= 0.0f ? 0 : (ss >= 255.0f ? 255 : (u8)(int)(ss + 0.5f));
      }
  }
  blend_into(im, deg, f);
}

// ---- geometry (NEAREST, fill 0) ----------------------------------------------------------------
// Image.transform(size, AFFINE, a): output pixel (x, y) samples input (a0 x' + a1 y' + a2,
// a3 x' + a4 y' + a5) at pixel centres x' = x + 0.5.  Pillow walks it in 16.16 fixed point
// (affine_fixed), or, for a pure scale / translation (a1 == a3 == 0), through a per-column table
// (ImagingScaleAffine).
void affine_nearest(Img& im, const double a[6]) {
  Img out = Img::zeros(im.w, im.h);  // the black fill
  const int W = im.w, H = im.h;
  if (a[1] == 0.0 && a[3] == 0.0) {
    std::vector<int> xin(W, -1);
    double xo = a[2] + a[0] * 0.5, yo = a[5] + a[4] * 0.5;
    for (int x = 0; x < W; ++x) {
      const int xi = xo < 0.0 ? -1 : (int)xo;
      xin[x] = (xi >= 0 && xi < W) ? xi : -1;
      xo += a[0];
    }
    for (int y = 0; y < H; ++y) {
      const int yi = yo < 0.0 ? -1 : (int)yo;
      if (yi >= 0 && yi < H) {
        const u8* src = im.row(yi);
        u8* dst = out.row(y);
        for (int x = 0; x < W; ++x)
          if (xin[x] >= 0) std::memcpy(dst + x * 3, src + xin[x] * 3, 3);
      }
      yo += a[4];
    }
  } else {
    auto fix = [](double v) { return (int)std::floor(v * 65536.0 + 0.5); };
    const int a0 = fix(a[0]), a1 = fix(a[1]), a3 = fix(a[3]), a4 = fix(a[4]);
    int a2 = fix(a[2] + a[1] * 0.5 + a[0] * 0.5), a5 = fix(a[5] + a[4] * 0.5 + a[3] * 0.5);
    for (int y = 0; y < H; ++y) {
      int xx = a2, yy = a5;
      u8* dst = out.row(y);
      for (int x = 0; x < W; ++x) {
        const int xi = xx >> 16, yi = yy >> 16;  // arithmetic shift = floor
        if (xi >= 0 && xi < W && yi >= 0 && yi < H) std::memcpy(dst + x * 3, im.row(yi) + xi * 3, 3);
        xx += a0;
        yy += a3;
      }
      a2 += a1;
      a5 += a4;
    }
  }
  im = std::move(out);
}

double py_round15(double v) {  // Python's round(v, 15): correctly rounded decimal, then back
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.15f", v);
  return std::strtod(buf, nullptr);
}

// Image.rotate(angle) (NEAREST, expand False, centre (w/2, h/2), fill 0)
void rotate(Img& im, double angle) {
  angle = std::fmod(angle, 360.0);
  if (angle < 0) angle += 360.0;  // Python's % takes the divisor's sign
  if (angle == 0.0) return;
  if (angle == 180.0) {  // Pillow's exact transpose (ROTATE_180)
    Img out(im.w, im.h);
    for (int y = 0; y < im.h; ++y)
      for (int x = 0; x < im.w; ++x) std::memcpy(out.row(im.h - 1 - y) + (im.w - 1 - x) * 3, im.row(y) + x * 3, 3);
    im = std::move(out);
    return;
  }
  if ((angle == 90.0 || angle == 270.0) && im.w == im.h) {
    Img out(im.w, im.h);
    const int n = im.w;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) {
        // ROTATE_90 (counter-clockwise): out(x', y') = in(n-1-y', x'); ROTATE_270: in(y', n-1-x')
        const int sx = angle == 90.0 ? n - 1 - y : y, sy = angle == 90.0 ? x : n - 1 - x;
        std::memcpy(out.row(y) + x * 3, im.row(sy) + sx * 3, 3);
      }
    im = std::move(out);
    return;
  }
  const double cx = im.w / 2.0, cy = im.h / 2.0;
  const double r = -(angle * (M_PI / 180.0));
  double m[6] = {py_round15(std::cos(r)), py_round15(std::sin(r)), 0.0, py_round15(-std::sin(r)),
                 py_round15(std::cos(r)), 0.0};
  const double tx = m[0] * (-cx) + m[1] * (-cy) + m[2], ty = m[3] * (-cx) + m[4] * (-cy) + m[5];
  m[2] = tx + cx;
  m[5] = ty + cy;
  affine_nearest(im, m);
}

// Cutout: ImageDraw.rectangle((x0, y0, x1, y1), fill) -- inclusive corners, clipped to the image
void fill_rect(Img& im, int x0, int y0, int x1, int y1, u8 v) {
  x0 = std::max(x0, 0);
  y0 = std::max(y0, 0);
  x1 = std::min(x1, im.w - 1);
  y1 = std::min(y1, im.h - 1);
  for (int y = y0; y <= y1; ++y) std::memset(im.row(y) + x0 * 3, v, (size_t)std::max(0, x1 - x0 + 1) * 3);
}

// CutoutAbs(img, v) (code/randaugment.py:47-60): centre uniform over [0, w) x [0, h)
void cutout_abs(Img& im, int v, Rng& rng) {
  const double fx = rng.uniform() * im.w, fy = rng.uniform() * im.h;
  const int x0 = (int)std::max(0.0, fx - v / 2.0), y0 = (int)std::max(0.0, fy - v / 2.0);
  const int x1 = (int)std::min((double)im.w, (double)x0 + v), y1 = (int)std::min((double)im.h, (double)y0 + v);
  fill_rect(im, x0, y0, x1, y1, 127);
}

// ---- resize (Image.resize(size, BILINEAR), Pillow's two-pass ImagingResample) -------------------
constexpr int PREC = 32 - 8 - 2;

struct Coeffs {
  int ksize = 0;
  std::vector<int> bounds;  // [out][2]: first input index, count
  std::vector<int> kk;      // [out][ksize]
};

Coeffs precompute(int in_size, int out_size) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  Coeffs c;
  c.ksize = (int)std::ceil(support) * 2 + 1;
  c.bounds.resize((size_t)out_size * 2);
  c.kk.assign((size_t)out_size * c.ksize, 0);
  std::vector<double> pre(c.ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double w = t < 1.0 ? 1.0 - t : 0.0;
      pre[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) pre[x] /= ww;
    for (int x = 0; x < c.ksize; ++x) {
      const double v = x < xmax ? pre[x] : 0.0;
      c.kk[(size_t)xx * c.ksize + x] = v < 0 ? (int)(-0.5 + v * (1 << PREC)) : (int)(0.5 + v * (1 << PREC));
    }
    c.bounds[xx * 2] = xmin;
    c.bounds[xx * 2 + 1] = xmax;
  }
  return c;
}

inline u8 clip8(int v) {
  v >>= PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : (u8)v);
}

// horizontal pass of rows [y0, y1) of src into dst (dst.w == ow)
template <class Src>
void resize_h(const Src& src, Img& dst, int ow) {
  const Coeffs c = precompute(src.w, ow);
  for (int y = 0; y < src.h; ++y) {
    const u8* s = src.row(y);
    u8* d = dst.row(y);
    for (int xx = 0; xx < ow; ++xx) {
      const int xmin = c.bounds[xx * 2], xmax = c.bounds[xx * 2 + 1];
      const int* k = &c.kk[(size_t)xx * c.ksize];
      int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
      for (int x = 0; x < xmax; ++x) {
        const u8* q = s + (x + xmin) * 3;
        s0 += q[0] * k[x];
        s1 += q[1] * k[x];
        s2 += q[2] * k[x];
      }
      d[xx * 3] = clip8(s0);
      d[xx * 3 + 1] = clip8(s1);
      d[xx * 3 + 2] = clip8(s2);
    }
  }
}

template <class Src>
void resize_v(const Src& src, Img& dst, int oh) {
  const Coeffs c = precompute(src.h, oh);
  const int rowb = src.w * 3;
  for (int yy = 0; yy < oh; ++yy) {
    const int ymin = c.bounds[yy * 2], ymax = c.bounds[yy * 2 + 1];
    const int* k = &c.kk[(size_t)yy * c.ksize];
    u8* d = dst.row(yy);
    for (int x = 0; x < rowb; ++x) {
      int a = 1 << (PREC - 1);
      for (int y = 0; y < ymax; ++y) a += src.row(y + ymin)[x] * k[y];
      d[x] = clip8(a);
    }
  }
}

// Image.resize((ow, oh), BILINEAR): horizontal pass first (over every row; Pillow restricts it to
// the rows the vertical pass reads -- the same values), then vertical; the source is read in place
Img resize_bilinear(const View& src, int ow, int oh) {
  if (ow == src.w && oh == src.h) {
    Img out(ow, oh);
    std::memcpy(out.px.data(), src.p, out.px.size());
    return out;
  }
  if (ow == src.w) {
    Img out(ow, oh);
    resize_v(src, out, oh);
    return out;
  }
  Img t(ow, src.h);
  resize_h(src, t, ow);
  if (oh == src.h) return t;
  Img out(ow, oh);
  resize_v(t, out, oh);
  return out;
}

// ---- crops / flips / padding ----------------------------------------------------------------------
Img crop(const Img& im, int left, int top, int cw, int ch) {  // inside the image
  Img out(cw, ch);
  for (int y = 0; y < ch; ++y) std::memcpy(out.row(y), im.row(top + y) + left * 3, (size_t)cw * 3);
  return out;
}

int py_round_half_even(double v) { return (int)std::nearbyint(v); }  // default rounding mode: ties to even

Img center_crop(const Img& im, int s) {  // torchvision F.center_crop (image at least s x s)
  const int top = py_round_half_even((im.h - s) / 2.0), left = py_round_half_even((im.w - s) / 2.0);
  return crop(im, left, top, s, s);
}

void hflip(Img& im) {
  for (int y = 0; y < im.h; ++y) {
    u8* r = im.row(y);
    for (int x = 0; x < im.w / 2; ++x)
      for (int c = 0; c < 3; ++c) std::swap(r[x * 3 + c], r[(im.w - 1 - x) * 3 + c]);
  }
}

void vflip(Img& im) {
  std::vector<u8> tmp((size_t)im.w * 3);
  for (int y = 0; y < im.h / 2; ++y) {
    std::memcpy(tmp.data(), im.row(y), tmp.size());
    std::memcpy(im.row(y), im.row(im.h - 1 - y), tmp.size());
    std::memcpy(im.row(im.h - 1 - y), tmp.data(), tmp.size());
  }
}

inline int reflect_idx(int i, int n) {  // numpy pad mode 'reflect' (edge not repeated), pad < n
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  i %= period;
  if (i < 0) i += period;
  return i < n ? i : period - i;
}

// RandomCrop(s, padding=pad, padding_mode='reflect'): pad every side, then crop at (top, left)
template <class Src>
Img pad_reflect_crop(const Src& im, int pad, int top, int left, int s) {
  Img out(s, s);
  for (int y = 0; y < s; ++y) {
    const int sy = reflect_idx(top + y - pad, im.h);
    for (int x = 0; x < s; ++x) std::memcpy(out.row(y) + x * 3, im.row(sy) + reflect_idx(left + x - pad, im.w) * 3, 3);
  }
  return out;
}

// ---- RandAugmentMC (code/randaugment.py:147-163, 207-222) --------------------------------------
enum Op {
  OP_AUTOCONTRAST = 0, OP_BRIGHTNESS, OP_COLOR, OP_CONTRAST, OP_EQUALIZE, OP_IDENTITY, OP_POSTERIZE, OP_ROTATE,
  OP_SHARPNESS, OP_SHEARX, OP_SHEARY, OP_SOLARIZE, OP_TRANSLATEX, OP_TRANSLATEY, OP_COUNT
};
// fixmatch_augment_pool(): (max_v, bias)
constexpr double POOL_MAX[OP_COUNT] = {0, 0.9, 0.9, 0.9, 0, 0, 4, 30, 0.9, 0.3, 0.3, 256, 0.3, 0.3};
constexpr double POOL_BIAS[OP_COUNT] = {0, 0.05, 0.05, 0.05, 0, 0, 4, 0, 0.05, 0, 0, 0, 0, 0};

double float_param(int v, double max_v) { return (double)v * max_v / 10.0; }   // _float_parameter
int int_param(int v, double max_v) { return (int)((double)v * max_v / 10.0); }  // _int_parameter

// one pool op at magnitude v; neg = the op's own random.random() < 0.5 sign draw (ops that have one)
void apply_op(Img& im, int op, int v, bool neg) {
  const double mx = POOL_MAX[op], bias = POOL_BIAS[op];
  switch (op) {
    case OP_AUTOCONTRAST: autocontrast(im); break;
    case OP_BRIGHTNESS: brightness(im, (float)(float_param(v, mx) + bias)); break;
    case OP_COLOR: color(im, (float)(float_param(v, mx) + bias)); break;
    case OP_CONTRAST: contrast(im, (float)(float_param(v, mx) + bias)); break;
    case OP_EQUALIZE: equalize(im); break;
    case OP_IDENTITY: break;
    case OP_POSTERIZE: posterize(im, int_param(v, mx) + (int)bias); break;
    case OP_ROTATE: {
      int a = int_param(v, mx) + (int)bias;
      rotate(im, neg ? -a : a);
      break;
    }
    case OP_SHARPNESS: sharpness(im, (float)(float_param(v, mx) + bias)); break;
    case OP_SHEARX: case OP_SHEARY: {
      double s = float_param(v, mx) + bias;
      if (neg) s = -s;
      const double m[6] = {1, op == OP_SHEARX ? s : 0, 0, op == OP_SHEARY ? s : 0, 1, 0};
      affine_nearest(im, m);
      break;
    }
    case OP_SOLARIZE: solarize(im, 256 - (int_param(v, mx) + (int)bias)); break;
    case OP_TRANSLATEX: case OP_TRANSLATEY: {
      double f = float_param(v, mx) + bias;
      if (neg) f = -f;
      const int t = (int)(f * (op == OP_TRANSLATEX ? im.w : im.h));
      const double m[6] = {1, 0, op == OP_TRANSLATEX ? (double)t : 0, 0, 1, op == OP_TRANSLATEY ? (double)t : 0};
      affine_nearest(im, m);
      break;
    }
    default: break;
  }
}

void randaugment_mc(Img& im, int n, int m, Rng& rng) {
  int ops[16];
  for (int i = 0; i < n && i < 16; ++i) ops[i] = rng.randint(0, OP_COUNT);  // random.choices(pool, k=n)
  for (int i = 0; i < n && i < 16; ++i) {
    const int v = rng.randint(1, m);  // np.random.randint(1, m)
    if (rng.uniform() < 0.5) {
      const bool neg = rng.uniform() < 0.5;
      apply_op(im, ops[i], v, neg);
    }
  }
  cutout_abs(im, (int)(32 * 0.5), rng);  // CutoutAbs(img, int(32 * 0.5))
}

// ---- the reference's composed transforms ------------------------------------------------------------
// TransformFixMatch (code/dataset.py:24-56): weak = Resize -> [CenterCrop]; strong = weak's resize /
// crop -> RandomHorizontalFlip -> RandomCrop(S, pad int(S * 0.125), reflect) -> RandAugmentMC(2, 10)
void to_chw(const Img& im, u8* dst);

void fixmatch_pair(const View& src, int S, bool is_crop, uint64_t seed, u8* weak_chw, u8* strong_chw) {
  const int R = is_crop ? (int)(S * 1.2) : S;
  Img base = resize_bilinear(src, R, R);
  if (is_crop) base = center_crop(base, S);
  to_chw(base, weak_chw);  // weak: no randomness
  Rng rng(seed);
  if (rng.uniform() < 0.5) hflip(base);  // the strong view continues from the same resize / crop
  const int pad = (int)(S * 0.125);
  const int top = rng.randint(0, 2 * pad + 1), left = rng.randint(0, 2 * pad + 1);
  Img strong = pad_reflect_crop(base, pad, top, left, S);
  randaugment_mc(strong, 2, 10, rng);
  to_chw(strong, strong_chw);
}

// The labeled train transform (code/dataset.py:185-196, IS_CROP): Resize(1.2 S) -> HFlip(0.3) ->
// VFlip(0.3) -> RandomRotation(20) -> CenterCrop(S) -> ColorJitter(brightness, contrast, saturation
// 0.2, in a random order) [-> ToTensor -> Normalize on the device]
void labeled_train(const View& src, int S, bool is_crop, uint64_t seed, Img& out) {
  const int R = is_crop ? (int)(S * 1.2) : S;
  Img im = resize_bilinear(src, R, R);
  Rng rng(seed);
  if (rng.uniform() < 0.3) hflip(im);
  if (rng.uniform() < 0.3) vflip(im);
  rotate(im, -20.0 + 40.0 * rng.uniform());  // uniform(-20, 20)
  im = center_crop(im, S);
  int order[3] = {0, 1, 2};
  for (int i = 2; i > 0; --i) std::swap(order[i], order[rng.randint(0, i + 1)]);
  for (int i = 0; i < 3; ++i) {
    const float f = (float)(0.8 + 0.4 * rng.uniform());  // uniform(0.8, 1.2)
    if (order[i] == 0) brightness(im, f);
    else if (order[i] == 1) contrast(im, f);
    else color(im, f);
  }
  out = std::move(im);
}

// ---- ColorJitter hue / RandomGrayscale (TransformCoMatch's strong_1) ------------------------------
// PIL's convert("HSV") / convert("RGB") from HSV (Convert.c, "following colorsys.py"): float / double
// arithmetic exactly as Pillow evaluates it, pinned by tests/test_host_aug.py.
inline void rgb2hsv_px(const u8* in, u8* out) {
  const u8 r = in[0], g = in[1], b = in[2];
  const u8 maxc = std::max(r, std::max(g, b)), minc = std::min(r, std::min(g, b));
  u8 uh = 0, us = 0;
  if (minc != maxc) {
    const float cr = (float)(maxc - minc);
    const float sat = cr / (float)maxc;
    const float rc = (float)(maxc - r) / cr, gc = (float)(maxc - g) / cr, bc = (float)(maxc - b) / cr;
    float h;
    if (r == maxc) h = bc - gc;
    else if (g == maxc) h = (float)(2.0 + rc - bc);
    else h = (float)(4.0 + gc - rc);
    h = (float)std::fmod(h / 6.0 + 1.0, 1.0);
    const int ih = (int)(h * 255.0), is = (int)(sat * 255.0);
    uh = (u8)(ih < 0 ? 0 : (ih > 255 ? 255 : ih));
    us = (u8)(is < 0 ? 0 : (is > 255 ? 255 : is));
  }
  out[0] = uh;
  out[1] = us;
  out[2] = maxc;
}

inline u8 clip_i(int v) { return (u8)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

inline void hsv2rgb_px(const u8* in, u8* out) {
  const u8 h = in[0], s = in[1], v = in[2];
  if (s == 0) {
    out[0] = out[1] = out[2] = v;
    return;
  }
  const int i = (int)std::floor((float)h * 6.0 / 255.0);
  const float f = (float)((float)h * 6.0 / 255.0 - (float)i);
  const float fs = (float)((float)s / 255.0);
  const u8 up = clip_i((int)std::round((float)v * (1.0 - fs)));
  const u8 uq = clip_i((int)std::round((float)v * (1.0 - fs * f)));
  const u8 ut = clip_i((int)std::round((float)v * (1.0 - fs * (1.0 - f))));
  switch (i % 6) {
    case 0: out[0] = v; out[1] = ut; out[2] = up; break;
    case 1: out[0] = uq; out[1] = v; out[2] = up; break;
    case 2: out[0] = up; out[1] = v; out[2] = ut; break;
    case 3: out[0] = up; out[1] = uq; out[2] = v; break;
    case 4: out[0] = ut; out[1] = up; out[2] = v; break;
    default: out[0] = v; out[1] = up; out[2] = uq; break;
  }
}

// torchvision adjust_hue on a PIL image: HSV, h += int8(hue_factor * 255) with uint8 wraparound, back
void adjust_hue(Img& im, double hue_factor) {
  const int shift = (int)(hue_factor * 255.0);  // np.int8(hue_factor * 255): truncation toward zero
  const size_t n = (size_t)im.w * im.h;
  u8 hsv[3];
  for (size_t i = 0; i < n; ++i) {
    u8* q = &im.px[i * 3];
    rgb2hsv_px(q, hsv);
    hsv[0] = (u8)((hsv[0] + shift) & 255);
    hsv2rgb_px(hsv, q);
  }
}

// rgb_to_grayscale(img, 3) on PIL: convert("L"), the gray replicated into three channels
void grayscale3(Img& im) {
  const size_t n = (size_t)im.w * im.h;
  for (size_t i = 0; i < n; ++i) {
    u8* q = &im.px[i * 3];
    q[0] = q[1] = q[2] = (u8)luma(q);
  }
}

void to_chw(const Img& im, u8* dst);

// TransformCoMatch (code/dataset.py:58-110, IS_CROP): weak = Resize -> CenterCrop -> HFlip; strong_0 =
// Resize -> CenterCrop -> HFlip -> RandAugmentMC(2, 10); strong_1 = Resize -> CenterCrop ->
// RandomApply([ColorJitter(0.4, 0.4, 0.4, 0.1)], p=0.8) -> RandomGrayscale(0.2) -> HFlip
void comatch_triplet(const View& src, int S, bool is_crop, uint64_t seed, u8* w_chw, u8* s0_chw, u8* s1_chw) {
  const int R = is_crop ? (int)(S * 1.2) : S;
  Img base = resize_bilinear(src, R, R);
  if (is_crop) base = center_crop(base, S);
  Rng rng(seed);
  {
    Img w = base;
    if (rng.uniform() < 0.5) hflip(w);
    to_chw(w, w_chw);
  }
  {
    Img s0 = base;
    if (rng.uniform() < 0.5) hflip(s0);
    randaugment_mc(s0, 2, 10, rng);
    to_chw(s0, s0_chw);
  }
  Img& s1 = base;
  if (rng.uniform() < 0.8) {  // ColorJitter: the four adjustments in a random order
    int order[4] = {0, 1, 2, 3};
    for (int i = 3; i > 0; --i) std::swap(order[i], order[rng.randint(0, i + 1)]);
    const float fb = (float)(0.6 + 0.8 * rng.uniform()), fc = (float)(0.6 + 0.8 * rng.uniform());
    const float fsat = (float)(0.6 + 0.8 * rng.uniform());
    const double fh = -0.1 + 0.2 * rng.uniform();
    for (int k = 0; k < 4; ++k) {
      if (order[k] == 0) brightness(s1, fb);
      else if (order[k] == 1) contrast(s1, fc);
      else if (order[k] == 2) color(s1, fsat);
      else adjust_hue(s1, fh);
    }
  }
  if (rng.uniform() < 0.2) grayscale3(s1);
  if (rng.uniform() < 0.5) hflip(s1);
  to_chw(s1, s1_chw);
}

// the validation / evaluation transform (code/dataset.py:217-231): Resize -> CenterCrop
void eval_view(const View& src, int S, bool is_crop, u8* chw) {
  const int R = is_crop ? (int)(S * 1.2) : S;
  Img base = resize_bilinear(src, R, R);
  if (is_crop) base = center_crop(base, S);
  to_chw(base, chw);
}

void to_chw(const Img& im, u8* dst) {  // planar [3][S][S]
  const size_t n = (size_t)im.w * im.h;
  for (size_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) dst[c * n + i] = im.px[i * 3 + c];
}

template <class F>
void parallel_for(int n, int nthreads, F f) {
  if (nthreads <= 1 || n <= 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> ts;
  const int T = std::min(nthreads, n);
  for (int t = 0; t < T; ++t)
    ts.emplace_back([&] {
      for (int i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& t : ts) t.join();
}

bool bad_img(const u8* p, int w, int h) { return !p || w <= 0 || h <= 0; }

}  // namespace

extern "C" {

// status codes shared with the device library (include/endossl.h)
enum { ESH_OK = 0, ESH_BAD_ARG = 2, ESH_BAD_SHAPE = 3 };

int esh_abi_version(void) { return 2; }

// One RandAugmentMC pool op on an RGB HWC image (src may equal dst): op index in
// fixmatch_augment_pool() order, magnitude v (1..10), neg = the op's sign draw.
int esh_aug_op(int op, const uint8_t* src, uint8_t* dst, int w, int h, int v, int neg) {
  if (bad_img(src, w, h) || !dst) return ESH_BAD_ARG;
  if (op < 0 || op >= OP_COUNT || v < 0 || v > 10) return ESH_BAD_ARG;
  Img im = from_ptr(src, w, h);
  apply_op(im, op, v, neg != 0);
  std::memcpy(dst, im.px.data(), im.px.size());
  return ESH_OK;
}

// ImageEnhance-style blend ops with an explicit factor: kind 0 brightness, 1 color, 2 contrast,
// 3 sharpness (ColorJitter and the pool ops share them).
int esh_enhance(int kind, const uint8_t* src, uint8_t* dst, int w, int h, float factor) {
  if (bad_img(src, w, h) || !dst || kind < 0 || kind > 3) return ESH_BAD_ARG;
  Img im = from_ptr(src, w, h);
  if (kind == 0) brightness(im, factor);
  else if (kind == 1) color(im, factor);
  else if (kind == 2) contrast(im, factor);
  else sharpness(im, factor);
  std::memcpy(dst, im.px.data(), im.px.size());
  return ESH_OK;
}

// Image.rotate(angle_deg) (NEAREST, no expand, fill 0)
// ColorJitter's hue adjustment (torchvision adjust_hue on PIL) and RandomGrayscale's 3-channel gray:
// kind 0 hue (factor in [-0.5, 0.5]), 1 grayscale (factor unused)
int esh_color_op(int kind, const uint8_t* src, uint8_t* dst, int w, int h, double factor) {
  if (bad_img(src, w, h) || !dst || kind < 0 || kind > 1 || (kind == 0 && !(factor >= -0.5 && factor <= 0.5)))
    return ESH_BAD_ARG;
  Img im = from_ptr(src, w, h);
  if (kind == 0) adjust_hue(im, factor);
  else grayscale3(im);
  std::memcpy(dst, im.px.data(), im.px.size());
  return ESH_OK;
}

int esh_rotate(const uint8_t* src, uint8_t* dst, int w, int h, double angle_deg) {
  if (bad_img(src, w, h) || !dst) return ESH_BAD_ARG;
  Img im = from_ptr(src, w, h);
  rotate(im, angle_deg);
  std::memcpy(dst, im.px.data(), im.px.size());
  return ESH_OK;
}

// Image.resize((ow, oh), BILINEAR)
int esh_resize_bilinear(const uint8_t* src, int w, int h, uint8_t* dst, int ow, int oh) {
  if (bad_img(src, w, h) || !dst || ow <= 0 || oh <= 0) return ESH_BAD_ARG;
  const Img out = resize_bilinear(View{src, w, h}, ow, oh);
  std::memcpy(dst, out.px.data(), out.px.size());
  return ESH_OK;
}

// CutoutAbs's rectangle: ImageDraw.rectangle((x0, y0, x1, y1), (v, v, v)), inclusive corners
int esh_fill_rect(uint8_t* img, int w, int h, int x0, int y0, int x1, int y1, int v) {
  if (bad_img(img, w, h) || v < 0 || v > 255) return ESH_BAD_ARG;
  Img im = from_ptr(img, w, h);
  fill_rect(im, x0, y0, x1, y1, (u8)v);
  std::memcpy(img, im.px.data(), im.px.size());
  return ESH_OK;
}

// RandomCrop(S, padding=pad, padding_mode='reflect') at a given offset: dst [S][S][3]
int esh_pad_reflect_crop(const uint8_t* src, int w, int h, int pad, int top, int left, int S, uint8_t* dst) {
  if (bad_img(src, w, h) || !dst || S <= 0 || pad < 0 || pad >= std::min(w, h) || top < 0 || left < 0 ||
      top + S > h + 2 * pad || left + S > w + 2 * pad)
    return ESH_BAD_SHAPE;
  const Img out = pad_reflect_crop(View{src, w, h}, pad, top, left, S);
  std::memcpy(dst, out.px.data(), out.px.size());
  return ESH_OK;
}

// Batch builders: images i = 0..n-1 (RGB HWC, sizes ws[i] x hs[i]), seeded per (seed, index), run on
// nthreads host threads; outputs planar uint8 [n][3][S][S] (es_patch_im2col_u8's input).
//  kind 0: TransformFixMatch -> weak (out0) and strong (out1)      code/dataset.py:24-56
//  kind 1: the labeled train transform -> out0 (out1 unused)      code/dataset.py:185-207
int esh_transform_batch(int kind, const uint8_t* const* srcs, const int* ws, const int* hs, int n, int S,
                        int is_crop, uint64_t seed, int nthreads, uint8_t* out0, uint8_t* out1, uint8_t* out2) {
  if (!srcs || !ws || !hs || n <= 0 || S <= 0 || !out0 || kind < 0 || kind > 3 || ((kind == 0 || kind == 2) && !out1) ||
      (kind == 2 && !out2))
    return ESH_BAD_ARG;
  const int R = is_crop ? (int)(S * 1.2) : S;
  for (int i = 0; i < n; ++i)
    if (bad_img(srcs[i], ws[i], hs[i]) || R < S) return ESH_BAD_SHAPE;
  const size_t per = (size_t)3 * S * S;
  parallel_for(n, nthreads, [&](int i) {
    const View src{srcs[i], ws[i], hs[i]};
    if (kind == 0) {
      fixmatch_pair(src, S, is_crop != 0, image_seed(seed, (uint64_t)i, 0), out0 + per * i, out1 + per * i);
    } else if (kind == 2) {
      comatch_triplet(src, S, is_crop != 0, image_seed(seed, (uint64_t)i, 2), out0 + per * i, out1 + per * i,
                      out2 + per * i);
    } else if (kind == 3) {
      eval_view(src, S, is_crop != 0, out0 + per * i);
    } else {
      Img out;
      labeled_train(src, S, is_crop != 0, image_seed(seed, (uint64_t)i, 1), out);
      to_chw(out, out0 + per * i);
    }
  });
  return ESH_OK;
}

}  // extern "C"
