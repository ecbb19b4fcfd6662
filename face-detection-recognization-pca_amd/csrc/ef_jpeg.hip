// Batched JPEG decode on the GPU ("batched JPEG decode -> gray ->
// resize"), feeding ef_preprocess without a host round trip.  Replaces the per-file
// cv2.imread of train-v4.py:59 (IMREAD_COLOR, then cvtColor + resize) and of
// useless/train.py:33 / scan-template-v4.py:52 (IMREAD_GRAYSCALE).
//
// Scope: baseline / extended sequential Huffman JPEG (SOF0/SOF1), 8-bit samples, one
// component (grey) or three (YCbCr, any of the sampling factors libjpeg accepts for which
// the luma has the maximal factors), one scan, optional restart intervals.  Progressive,
// arithmetic-coded, 12-bit, CMYK/Adobe-RGB and multi-scan files are reported unsupported
// per image (status < 0) and the caller decodes them on the host.
//
// Arithmetic restated from libjpeg-turbo (what both OpenCV's imread and Pillow link), the
// library's defaults (JDCT_ISLOW, fancy upsampling):
//   * entropy decoding: jdhuff.c (8-bit lookahead tables, HUFF_EXTEND, 0xFF00 stuffing, a
//     marker ends the data and zeros are fed, restart markers reset the DC predictors);
//   * inverse DCT: jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2, the all-zero
//     column / row shortcuts, range_limit[x & RANGE_MASK] output);
//   * grey output from YCbCr: component 0 (jdcolor.c grayscale_convert);
//   * colour: jdsample.c h2v1 / h2v2 fancy (triangle) upsampling with libjpeg's edge
//     replication, jdcolor.c ycc_rgb_convert with its SCALEBITS 16 tables, emitted as BGR
//     (cv2.imread's channel order).
// The restatement is pinned bit for bit against Pillow's libjpeg-turbo decode in
// tests/test_gpu_jpeg.py (grey and colour, 4:4:4 / 4:2:2 / 4:2:0, odd sizes, restart
// intervals, several qualities).
//
// Work split: the host parses the markers (tables, frame, scan, restart segments); kernel 1
// decodes one entropy segment per thread (a whole scan, or one restart interval) into
// int16 coefficient blocks; kernel 2 runs one 8x8 IDCT per thread into padded component
// planes; kernel 3 writes one output pixel per thread (grey copy, or upsample + YCC->BGR).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ef_internal.hpp"

namespace ef {
namespace {

constexpr int kMaxComp = 3;

struct HuffTab {                // libjpeg d_derived_tbl
  unsigned short look[256];     // (nbits << 8) | symbol for codes <= 8 bits; nbits 0 = longer
  int maxcode[18];              // largest code of each length (-1: none), maxcode[17] sentinel
  int valoffset[18];            // huffval index offset per length
  unsigned char huffval[256];
};

struct JComp {
  int h, v;          // sampling factors
  int q;             // quantisation table index into the image's qt[]
  int dc, ac;        // Huffman table indices into the global pool
  int bw, bh;        // blocks per row / column in the coefficient & sample planes
  int dw, dh;        // downsampled width / height (libjpeg's downsampled_width/height)
  int64_t coef_off;  // first block's int16[64] in the coefficient buffer
  int64_t plane_off; // first sample of the padded plane (bw * 8 bytes per row)
};

struct JImage {
  int w, h, nc, hmax, vmax;
  int mcux, mcuy;          // MCUs per row / column (interleaved), or blocks (one component)
  int interleaved;
  int restart;             // MCUs per restart interval (0 = none)
  int qt_base;             // first of this image's quantisation tables (4 slots) in the pool
  JComp c[kMaxComp];
  int64_t out_off;
  int mode;                // EF_JPEG_GRAY / EF_JPEG_BGR
};

struct JSeg {
  int img;
  int64_t beg, end;  // entropy-coded bytes [beg, end) in the uploaded data
  int mcu0, nmcu;    // first MCU and count
};

// --------------------------------------------------------------------- host parsing
struct RawHuff {
  unsigned char bits[17];
  unsigned char val[256];
  bool present = false;
};

bool derive(const RawHuff& r, HuffTab& t) {  // jdhuff.c jpeg_make_d_derived_tbl
  char size[257];
  unsigned code[257];
  int p = 0;
  for (int l = 1; l <= 16; ++l) {
    int n = r.bits[l];
    if (p + n > 256) return false;
    while (n--) size[p++] = (char)l;
  }
  size[p] = 0;
  const int last = p;
  unsigned cd = 0;
  int si = size[0];
  p = 0;
  while (size[p]) {
    while ((int)size[p] == si) code[p++] = cd++;
    if (cd >= (1u << si)) return false;
    cd <<= 1;
    si++;
  }
  p = 0;
  for (int l = 1; l <= 16; ++l) {
    if (r.bits[l]) {
      t.valoffset[l] = p - (int)code[p];
      p += r.bits[l];
      t.maxcode[l] = (int)code[p - 1];
    } else {
      t.maxcode[l] = -1;
    }
  }
  t.valoffset[17] = 0;
  t.maxcode[17] = 0x7FFFFFFF;  // sentinel: ensures the slow decode terminates
  t.maxcode[0] = -1;
  t.valoffset[0] = 0;
  for (int i = 0; i < 256; ++i) t.look[i] = 0;
  p = 0;
  for (int l = 1; l <= 8; ++l)
    for (int i = 1; i <= r.bits[l]; ++i, ++p) {
      int lookbits = (int)code[p] << (8 - l);
      for (int ctr = 1 << (8 - l); ctr > 0; --ctr) t.look[lookbits++] = (unsigned short)((l << 8) | r.val[p]);
    }
  for (int i = 0; i < 256; ++i) t.huffval[i] = i < last ? r.val[i] : 0;
  return true;
}

// Parse one file: frame, tables, scan, restart segments.  Returns 0 or a negative status.
int parse(const uint8_t* d, int64_t n, int img_index, JImage& im, std::vector<HuffTab>& pool,
          std::vector<unsigned short>& qpool, std::vector<JSeg>& segs, int64_t data_base, bool want) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return EF_JPEG_E_CORRUPT;
  RawHuff dht[2][4];
  unsigned short qt[4][64];
  bool qt_ok[4] = {false, false, false, false};
  int comp_id[kMaxComp] = {0, 0, 0};
  int comp_q[kMaxComp] = {0, 0, 0};
  bool have_frame = false;
  bool jfif = false;
  int adobe_transform = -1;
  im.restart = 0;
  int64_t p = 2;
  static const unsigned char zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                       12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                       35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                       58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
  while (p + 4 <= n) {
    if (d[p] != 0xFF) return EF_JPEG_E_CORRUPT;
    const int m = d[p + 1];
    if (m == 0xFF) { ++p; continue; }  // fill byte
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) { p += 2; continue; }
    if (m == 0xD9) return EF_JPEG_E_CORRUPT;  // EOI before any scan
    const int len = (d[p + 2] << 8) | d[p + 3];
    if (len < 2 || p + 2 + len > n) return EF_JPEG_E_CORRUPT;
    const uint8_t* s = d + p + 4;
    const int sl = len - 2;
    if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential Huffman
      if (sl < 6 || s[0] != 8) return EF_JPEG_E_UNSUPPORTED;
      im.h = (s[1] << 8) | s[2];
      im.w = (s[3] << 8) | s[4];
      im.nc = s[5];
      if (im.w <= 0 || im.h <= 0 || (im.nc != 1 && im.nc != 3) || sl < 6 + 3 * im.nc) return EF_JPEG_E_UNSUPPORTED;
      im.hmax = im.vmax = 1;
      for (int c = 0; c < im.nc; ++c) {
        comp_id[c] = s[6 + 3 * c];
        im.c[c].h = s[7 + 3 * c] >> 4;
        im.c[c].v = s[7 + 3 * c] & 15;
        comp_q[c] = s[8 + 3 * c];
        if (im.c[c].h < 1 || im.c[c].h > 4 || im.c[c].v < 1 || im.c[c].v > 4 || comp_q[c] > 3)
          return EF_JPEG_E_CORRUPT;
        im.hmax = std::max(im.hmax, im.c[c].h);
        im.vmax = std::max(im.vmax, im.c[c].v);
      }
      have_frame = true;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return EF_JPEG_E_UNSUPPORTED;  // progressive, lossless, arithmetic, hierarchical
    } else if (m == 0xC4) {  // DHT
      int q = 0;
      while (q < sl) {
        if (q + 17 > sl) return EF_JPEG_E_CORRUPT;
        const int tc = s[q] >> 4, th = s[q] & 15;
        if (tc > 1 || th > 3) return EF_JPEG_E_CORRUPT;
        RawHuff& r = dht[tc][th];
        int cnt = 0;
        r.bits[0] = 0;
        for (int l = 1; l <= 16; ++l) cnt += (r.bits[l] = s[q + l]);
        if (cnt > 256 || q + 17 + cnt > sl) return EF_JPEG_E_CORRUPT;
        std::memcpy(r.val, s + q + 17, cnt);
        for (int i = cnt; i < 256; ++i) r.val[i] = 0;
        r.present = true;
        q += 17 + cnt;
      }
    } else if (m == 0xDB) {  // DQT
      int q = 0;
      while (q < sl) {
        const int pq = s[q] >> 4, tq = s[q] & 15;
        if (tq > 3 || pq > 1 || q + 1 + 64 * (pq + 1) > sl) return EF_JPEG_E_CORRUPT;
        for (int i = 0; i < 64; ++i)
          qt[tq][zz[i]] = pq ? (unsigned short)((s[q + 1 + 2 * i] << 8) | s[q + 2 + 2 * i]) : s[q + 1 + i];
        qt_ok[tq] = true;
        q += 1 + 64 * (pq + 1);
      }
    } else if (m == 0xE0) {  // APP0: JFIF means YCbCr (jdmarker.c examine_app0)
      if (sl >= 5 && std::memcmp(s, "JFIF", 5) == 0) jfif = true;
    } else if (m == 0xEE) {  // APP14: Adobe colour transform (examine_app14)
      if (sl >= 12 && std::memcmp(s, "Adobe", 5) == 0) adobe_transform = s[11];
    } else if (m == 0xDD) {  // DRI
      if (sl < 2) return EF_JPEG_E_CORRUPT;
      im.restart = (s[0] << 8) | s[1];
    } else if (m == 0xDA) {  // SOS: the (single) scan
      if (!have_frame || sl < 1) return EF_JPEG_E_CORRUPT;
      const int ns = s[0];
      if (ns != im.nc || sl < 1 + 2 * ns + 3) return EF_JPEG_E_UNSUPPORTED;  // multi-scan sequential
      int map_dc[4] = {-1, -1, -1, -1}, map_ac[4] = {-1, -1, -1, -1};
      for (int k = 0; k < ns; ++k) {
        const int cid = s[1 + 2 * k], td = s[2 + 2 * k] >> 4, ta = s[2 + 2 * k] & 15;
        int c = -1;
        for (int j = 0; j < im.nc; ++j)
          if (comp_id[j] == cid) c = j;
        if (c != k || td > 3 || ta > 3 || !dht[0][td].present || !dht[1][ta].present) return EF_JPEG_E_CORRUPT;
        if (map_dc[td] < 0) {
          map_dc[td] = (int)pool.size();
          pool.emplace_back();
          if (!derive(dht[0][td], pool.back())) return EF_JPEG_E_CORRUPT;
        }
        if (map_ac[ta] < 0) {
          map_ac[ta] = (int)pool.size();
          pool.emplace_back();
          if (!derive(dht[1][ta], pool.back())) return EF_JPEG_E_CORRUPT;
        }
        im.c[c].dc = map_dc[td];
        im.c[c].ac = map_ac[ta];
        if (!qt_ok[comp_q[c]]) return EF_JPEG_E_CORRUPT;
      }
      const int ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahal = s[3 + 2 * ns];
      if (ss != 0 || se != 63 || ahal != 0) return EF_JPEG_E_UNSUPPORTED;
      // colour space (jdapimin.c default_decompress_parms): only YCbCr is restated
      if (im.nc == 3 && !jfif) {
        const bool rgb_ids = comp_id[0] == 'R' && comp_id[1] == 'G' && comp_id[2] == 'B';
        if (adobe_transform == 0 || (adobe_transform < 0 && rgb_ids)) return EF_JPEG_E_UNSUPPORTED;
      }
      // geometry (jdinput.c initial_setup / per_scan_setup)
      im.interleaved = im.nc > 1;
      if (im.nc == 3 && (im.c[0].h != im.hmax || im.c[0].v != im.vmax)) return EF_JPEG_E_UNSUPPORTED;
      for (int c = 0; c < im.nc; ++c) {
        const int hm = im.hmax, vm = im.vmax;
        // only the factors libjpeg-turbo's fancy upsamplers handle are restated
        if (c > 0 && !((hm == im.c[c].h || hm == 2 * im.c[c].h) && (vm == im.c[c].v || vm == 2 * im.c[c].v)))
          return EF_JPEG_E_UNSUPPORTED;
        if (c > 0 && vm == 2 * im.c[c].v && hm != 2 * im.c[c].h) return EF_JPEG_E_UNSUPPORTED;  // h1v2
        im.c[c].dw = (int)(((int64_t)im.w * im.c[c].h + hm - 1) / hm);
        im.c[c].dh = (int)(((int64_t)im.h * im.c[c].v + vm - 1) / vm);
      }
      if (im.interleaved) {
        im.mcux = (im.w + 8 * im.hmax - 1) / (8 * im.hmax);
        im.mcuy = (im.h + 8 * im.vmax - 1) / (8 * im.vmax);
        for (int c = 0; c < im.nc; ++c) {
          im.c[c].bw = im.mcux * im.c[c].h;
          im.c[c].bh = im.mcuy * im.c[c].v;
        }
      } else {
        im.c[0].bw = (im.c[0].dw + 7) / 8;
        im.c[0].bh = (im.c[0].dh + 7) / 8;
        im.mcux = im.c[0].bw;
        im.mcuy = im.c[0].bh;
      }
      im.qt_base = (int)(qpool.size() / 64);
      for (int c = 0; c < im.nc; ++c) {
        qpool.insert(qpool.end(), qt[comp_q[c]], qt[comp_q[c]] + 64);
        im.c[c].q = c;
      }
      if (!want) return 0;
      // entropy segments: the scan data up to the next non-RST marker, split at RSTn
      const int64_t scan_beg = p + 2 + len;
      const int64_t total_mcu = (int64_t)im.mcux * im.mcuy;
      int64_t q = scan_beg, seg_beg = scan_beg;
      int mcu0 = 0;
      const int per = im.restart > 0 ? im.restart : (int)std::min<int64_t>(total_mcu, 0x7FFFFFFF);
      while (true) {
        if (q + 1 >= n) break;  // truncated: the last segment runs to the end (zeros fed)
        if (d[q] == 0xFF && d[q + 1] != 0x00 && d[q + 1] != 0xFF) {
          const int mk = d[q + 1];
          if (im.restart > 0 && mk >= 0xD0 && mk <= 0xD7) {
            const int cnt = (int)std::min<int64_t>(per, total_mcu - mcu0);
            if (cnt > 0) segs.push_back(JSeg{img_index, data_base + seg_beg, data_base + q, mcu0, cnt});
            mcu0 += cnt;
            q += 2;
            seg_beg = q;
            continue;
          }
          break;
        }
        ++q;
      }
      const int64_t seg_end = std::min<int64_t>(q + (q + 1 >= n ? 1 : 0), n);
      if (mcu0 < total_mcu) {
        const int cnt = (int)(total_mcu - mcu0);
        // libjpeg's decoder keeps decoding MCUs past a missing RST with zeros fed; one
        // segment covers every remaining MCU (restart interval boundaries inside it
        // reset the predictors as the stream would)
        segs.push_back(JSeg{img_index, data_base + seg_beg, data_base + seg_end, mcu0, cnt});
      }
      return 0;
    }
    p += 2 + len;
  }
  return EF_JPEG_E_CORRUPT;
}

// ------------------------------------------------------------------------ kernels
#define EF_NATURAL_ORDER \
  {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,   \
   6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,   \
   39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63}
// zigzag -> natural order, padded with 63 for the k += r overrun of a corrupt stream (jutils.c)
__constant__ unsigned char kNatural[80] = EF_NATURAL_ORDER;
#ifdef EF_DIAGNOSTICS
const unsigned char kNaturalHost[80] = EF_NATURAL_ORDER;
#endif

struct BitReader {  // jdhuff.c bit buffer; a marker or the segment end feeds zeros
  const uint8_t* p;
  const uint8_t* end;
  unsigned long long buf;
  int bits;
  __host__ __device__ void fill() {
    while (bits <= 56) {
      unsigned c = 0;
      if (p < end) {
        c = *p;
        if (c == 0xFF) {
          const unsigned nx = p + 1 < end ? p[1] : 0xD9u;
          if (nx == 0x00) {
            p += 2;
          } else {  // a marker: stop, feed zeros
            end = p;
            c = 0;
          }
        } else {
          ++p;
        }
      }
      buf |= (unsigned long long)c << (56 - bits);
      bits += 8;
    }
  }
  __host__ __device__ unsigned peek(int n) { return (unsigned)(buf >> (64 - n)); }
  __host__ __device__ void skip(int n) { buf <<= n; bits -= n; }
  __host__ __device__ int get(int n) {  // n <= 16
    if (n == 0) return 0;
    if (bits < n) fill();
    const int v = (int)peek(n);
    skip(n);
    return v;
  }
  __host__ __device__ int decode(const HuffTab& t) {
    if (bits < 16) fill();
    const unsigned look = peek(8);
    const unsigned e = t.look[look];
    if (e >> 8) {
      skip((int)(e >> 8));
      return (int)(e & 0xFF);
    }
    int l = 9;
    int code = (int)peek(9);
    while (l <= 16 && code > t.maxcode[l]) {
      ++l;
      code = (int)peek(l);
    }
    if (l > 16) {  // corrupt: libjpeg warns and returns 0
      skip(16);
      return 0;
    }
    skip(l);
    return t.huffval[(code + t.valoffset[l]) & 0xFF];
  }
};

__host__ __device__ __forceinline__ int huff_extend(int x, int s) { return x < (1 << (s - 1)) ? x + (-1 << s) + 1 : x; }

// One entropy segment (a whole scan, or one restart interval) -> int16 coefficient blocks.
__host__ __device__ void huff_segment(const uint8_t* data, const JSeg& sg, const JImage& im, const HuffTab* pool,
                                      short* coef, const unsigned char* nat) {
  BitReader br{data + sg.beg, data + sg.end, 0ull, 0};
  br.fill();
  int pred[kMaxComp] = {0, 0, 0};
  for (int t = 0; t < sg.nmcu; ++t) {
    const int mcu = sg.mcu0 + t;
    if (im.restart > 0 && t > 0 && mcu % im.restart == 0) {  // a restart boundary without RSTn
      pred[0] = pred[1] = pred[2] = 0;
      br.skip(br.bits & 7);
    }
    const int my = mcu / im.mcux, mx = mcu - my * im.mcux;
    for (int c = 0; c < im.nc; ++c) {
      const JComp& cp = im.c[c];
      const int nby = im.interleaved ? cp.v : 1, nbx = im.interleaved ? cp.h : 1;
      for (int yy = 0; yy < nby; ++yy)
        for (int xx = 0; xx < nbx; ++xx) {
          const int by = im.interleaved ? my * cp.v + yy : my, bx = im.interleaved ? mx * cp.h + xx : mx;
          short* blk = coef + cp.coef_off + ((int64_t)by * cp.bw + bx) * 64;
          for (int i = 0; i < 64; ++i) blk[i] = 0;
          int s = br.decode(pool[cp.dc]);
          if (s) s = huff_extend(br.get(s), s);
          pred[c] += s;
          blk[0] = (short)pred[c];
          const HuffTab& at = pool[cp.ac];
          for (int k = 1; k < 64; ++k) {
            int r = br.decode(at);
            s = r & 15;
            r >>= 4;
            if (s) {
              k += r;
              const int v = huff_extend(br.get(s), s);
              blk[nat[k]] = (short)v;
            } else {
              if (r != 15) break;
              k += 15;
            }
          }
        }
    }
  }
}

__global__ __launch_bounds__(64) void jpeg_huff_kernel(const uint8_t* __restrict__ data, const JSeg* __restrict__ segs,
                                                      int nseg, const JImage* __restrict__ imgs,
                                                      const HuffTab* __restrict__ pool, short* __restrict__ coef) {
  const int si = blockIdx.x * blockDim.x + threadIdx.x;
  if (si >= nseg) return;
  const JSeg sg = segs[si];
  huff_segment(data, sg, imgs[sg.img], pool, coef, kNatural);
}

// jidctint.c jpeg_idct_islow arithmetic
constexpr int CB = 13, P1 = 2;
__host__ __device__ __forceinline__ int descale(long long x, int n) { return (int)((x + (1LL << (n - 1))) >> n); }
__host__ __device__ __forceinline__ unsigned char range_limit(int x) {  // sample_range_limit + CENTERJSAMPLE, idx & 1023
  const int i = x & 1023;
  if (i < 128) return (unsigned char)(i + 128);
  if (i < 512) return 255;
  if (i < 896) return 0;
  return (unsigned char)(i - 896);
}

// One islow 1-D pass over (i0..i7); o[] receives the eight sums before descaling, in the
// output order 0..7 (jidctint.c's "Final output stage").
__host__ __device__ __forceinline__ void islow_1d(long long i0, long long i1, long long i2, long long i3, long long i4,
                                         long long i5, long long i6, long long i7, long long o[8]) {
  long long z2 = i2, z3 = i6;
  long long z1 = (z2 + z3) * 4433;             // FIX_0_541196100
  long long tmp2 = z1 + z3 * -15137;           // FIX_1_847759065
  long long tmp3 = z1 + z2 * 6270;             // FIX_0_765366865
  long long tmp0 = (i0 + i4) * (1LL << CB);
  long long tmp1 = (i0 - i4) * (1LL << CB);
  const long long tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  tmp0 = i7;
  tmp1 = i5;
  tmp2 = i3;
  tmp3 = i1;
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  long long z4 = tmp1 + tmp3;
  const long long z5 = (z3 + z4) * 9633;  // FIX_1_175875602
  tmp0 *= 2446;                           // FIX_0_298631336
  tmp1 *= 16819;                          // FIX_2_053119869
  tmp2 *= 25172;                          // FIX_3_072711026
  tmp3 *= 12299;                          // FIX_1_501321110
  z1 *= -7373;                            // FIX_0_899976223
  z2 *= -20995;                           // FIX_2_562915447
  z3 *= -16069;                           // FIX_1_961570560
  z4 *= -3196;                            // FIX_0_390180644
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  o[0] = tmp10 + tmp3;
  o[7] = tmp10 - tmp3;
  o[1] = tmp11 + tmp2;
  o[6] = tmp11 - tmp2;
  o[2] = tmp12 + tmp1;
  o[5] = tmp12 - tmp1;
  o[3] = tmp13 + tmp0;
  o[4] = tmp13 - tmp0;
}

// pass 1 of block `in` (dequantised by q) on column j into the workspace w[64]
__host__ __device__ __forceinline__ void idct_col(const short* in, const unsigned short* q, int j, int* w) {
  long long v[8];
  bool ac0 = true;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    v[r] = (long long)in[8 * r + j] * q[8 * r + j];
    if (r > 0 && in[8 * r + j] != 0) ac0 = false;
  }
  if (ac0) {
    const int dcval = (int)(v[0] * (1 << P1));
#pragma unroll
    for (int r = 0; r < 8; ++r) w[8 * r + j] = dcval;
  } else {
    long long o[8];
    islow_1d(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], o);
#pragma unroll
    for (int r = 0; r < 8; ++r) w[8 * r + j] = descale(o[r], CB - P1);
  }
}

// pass 2 on row j of the workspace: the row's 8 samples packed little-endian
__host__ __device__ __forceinline__ unsigned long long idct_row(const int* w, int j) {
  const int* rw = w + 8 * j;
  unsigned char o8[8];
  if (rw[1] == 0 && rw[2] == 0 && rw[3] == 0 && rw[4] == 0 && rw[5] == 0 && rw[6] == 0 && rw[7] == 0) {
    const unsigned char v = range_limit(descale((long long)rw[0], P1 + 3));
#pragma unroll
    for (int c = 0; c < 8; ++c) o8[c] = v;
  } else {
    long long o[8];
    islow_1d(rw[0], rw[1], rw[2], rw[3], rw[4], rw[5], rw[6], rw[7], o);
#pragma unroll
    for (int c = 0; c < 8; ++c) o8[c] = range_limit(descale(o[c], CB + P1 + 3));
  }
  unsigned long long packed = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) packed |= (unsigned long long)o8[c] << (8 * c);
  return packed;
}

// jidctint.c jpeg_idct_islow with eight lanes per 8x8 block: lane j runs pass 1 on column j
// and, after an exchange through LDS, pass 2 on row j, storing its 8 samples as one 64-bit
// write into the padded component plane.  The eight lanes of a block share a wave.
constexpr int kIdctBlocks = 32;  // blocks per 256-thread workgroup
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const short* __restrict__ coef, const JImage* __restrict__ imgs,
                                                       const int64_t* __restrict__ block_start, int nruns,
                                                       const int* __restrict__ ic_img, const unsigned short* __restrict__ qpool,
                                                       int64_t total_blocks, uint8_t* __restrict__ planes) {
  __shared__ int ws[kIdctBlocks][65];
  const int lb = threadIdx.x >> 3, j = threadIdx.x & 7;
  const int64_t gb = (int64_t)blockIdx.x * kIdctBlocks + lb;
  if (gb >= total_blocks) return;  // whole 8-lane groups leave together
  int lo = 0, hi = nruns - 1;  // the (image, component) run holding this block
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_start[mid] <= gb) lo = mid; else hi = mid - 1;
  }
  const int img = ic_img[lo] >> 2, comp = ic_img[lo] & 3;
  const JImage& im = imgs[img];
  const JComp& cp = im.c[comp];
  const int64_t b = gb - block_start[lo];
  const int by = (int)(b / cp.bw), bx = (int)(b - (int64_t)by * cp.bw);
  const short* in = coef + cp.coef_off + b * 64;
  const unsigned short* q = qpool + (int64_t)(im.qt_base + cp.q) * 64;
  int* w = ws[lb];
  idct_col(in, q, j, w);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are visible
  __builtin_amdgcn_wave_barrier();
  const unsigned long long packed = idct_row(w, j);
  const int64_t pitch = (int64_t)cp.bw * 8;
  *reinterpret_cast<unsigned long long*>(planes + cp.plane_off + ((int64_t)by * 8 + j) * pitch + (int64_t)bx * 8) = packed;
}

// jdcolor.c build_ycc_rgb_table
__host__ __device__ __forceinline__ int cr_r(int cr) { return (91881 * (cr - 128) + 32768) >> 16; }
__host__ __device__ __forceinline__ int cb_b(int cb) { return (116130 * (cb - 128) + 32768) >> 16; }
__host__ __device__ __forceinline__ int cbcr_g(int cb, int cr) {
  return ((-22554) * (cb - 128) + 32768 + (-46802) * (cr - 128)) >> 16;
}
__host__ __device__ __forceinline__ unsigned char clamp255(int x) { return (unsigned char)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

// jdsample.c fancy upsampling of a chroma sample at output (y, x) of component cp.  Column
// dw is taken as a copy of column dw-1, as libjpeg-turbo's SIMD upsamplers (the x86-64 build
// both OpenCV and Pillow ship) insert it; this differs from the C fallback only when dw == 1.
__host__ __device__ int upsample(const uint8_t* pl, const JComp& cp, int hmax, int vmax, int y, int x) {
  const int64_t pitch = (int64_t)cp.bw * 8;
  const bool h2 = hmax == 2 * cp.h, v2 = vmax == 2 * cp.v;
  if (!h2 && !v2) return pl[(int64_t)y * pitch + x];
  const int j = h2 ? x >> 1 : x, u = x & 1;
  // jdsample.c jinit_upsampler: fancy only when downsampled_width > 2, else box replication
  if (cp.dw <= 2) return pl[(int64_t)(v2 ? y >> 1 : y) * pitch + j];
  if (!v2) {  // h2v1_fancy_upsample
    const uint8_t* r = pl + (int64_t)y * pitch;
    if (u == 0) return j == 0 ? r[0] : (r[j] * 3 + r[j - 1] + 1) >> 2;
    if (j == cp.dw - 1) return r[j];
    return (r[j] * 3 + r[j + 1] + 2) >> 2;
  }
  // h2v2_fancy_upsample; rows above the first / below the last replicate them
  const int i = y >> 1, v = y & 1;
  int i1 = v == 0 ? i - 1 : i + 1;
  i1 = i1 < 0 ? 0 : (i1 > cp.dh - 1 ? cp.dh - 1 : i1);
  const uint8_t* r0 = pl + (int64_t)i * pitch;
  const uint8_t* r1 = pl + (int64_t)i1 * pitch;
  auto cs = [&](int c) { return r0[c] * 3 + r1[c]; };
  if (u == 0) return j == 0 ? (cs(0) * 4 + 8) >> 4 : (cs(j) * 3 + cs(j - 1) + 8) >> 4;
  if (j == cp.dw - 1) return (cs(j) * 4 + 7) >> 4;
  return (cs(j) * 3 + cs(j + 1) + 7) >> 4;
}

// output pixel k (raster order) of image im: grey copy, grey->BGR, or upsample + YCC->BGR
__host__ __device__ void out_pixel(const JImage& im, int64_t k, const uint8_t* planes, uint8_t* out) {
  const int y = (int)(k / im.w), x = (int)(k - (int64_t)y * im.w);
  const uint8_t* p0 = planes + im.c[0].plane_off;
  const int Y = p0[(int64_t)y * im.c[0].bw * 8 + x];
  if (im.mode == EF_JPEG_GRAY) {
    out[im.out_off + k] = (uint8_t)Y;
    return;
  }
  uint8_t* o = out + im.out_off + 3 * k;
  if (im.nc == 1) {  // gray_rgb_convert
    o[0] = o[1] = o[2] = (uint8_t)Y;
    return;
  }
  const int cb = upsample(planes + im.c[1].plane_off, im.c[1], im.hmax, im.vmax, y, x);
  const int cr = upsample(planes + im.c[2].plane_off, im.c[2], im.hmax, im.vmax, y, x);
  o[0] = clamp255(Y + cb_b(cb));       // B
  o[1] = clamp255(Y + cbcr_g(cb, cr));  // G
  o[2] = clamp255(Y + cr_r(cr));       // R
}

__global__ __launch_bounds__(256) void jpeg_out_kernel(const JImage* __restrict__ imgs, const int64_t* __restrict__ px_start,
                                                      int nimg, int64_t total_px, const uint8_t* __restrict__ planes,
                                                      uint8_t* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total_px) return;
  int lo = 0, hi = nimg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (px_start[mid] <= g) lo = mid; else hi = mid - 1;
  }
  out_pixel(imgs[lo], g - px_start[lo], planes, out);
}

// ------------------------------------------------------------------ batch layout
// Everything one decode launch needs, built on the host: per-image geometry, Huffman and
// quantisation tables, entropy segments, IDCT runs and output pixel starts.
struct Batch {
  std::vector<HuffTab> pool;
  std::vector<unsigned short> qpool;
  std::vector<JSeg> segs;
  std::vector<JImage> imgs;
  std::vector<int> img_of;            // input index of each decoded image
  std::vector<int64_t> block_start;   // IDCT runs: first global block of (image, component)
  std::vector<int> ic;                // (image << 2) | component of each run
  std::vector<int64_t> px_start;      // first output pixel of each image
  int64_t data_bytes = 0, coef_blocks = 0, plane_bytes = 0, blocks = 0, pixels = 0, dense_out = 0;
};

// dev_out: images land at out_offsets (device layout); otherwise packed densely
void build_batch(const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int count, int mode,
                 const int64_t* out_offsets, int32_t* status, Batch& B) {
  const int ch = mode == EF_JPEG_GRAY ? 1 : 3;
  for (int i = 0; i < count; ++i) {
    JImage im{};
    const size_t seg0 = B.segs.size(), pool0 = B.pool.size(), q0 = B.qpool.size();
    int st = sizes[i] > 0 ? parse(data + offsets[i], sizes[i], (int)B.imgs.size(), im, B.pool, B.qpool, B.segs,
                                  B.data_bytes, true)
                          : EF_JPEG_E_CORRUPT;
    if (st == 0 && (int64_t)im.w * im.h > ((int64_t)1 << 31)) st = EF_JPEG_E_UNSUPPORTED;
    if (status) status[i] = st;
    if (st != 0) {
      B.segs.resize(seg0);
      B.pool.resize(pool0);
      B.qpool.resize(q0);
      continue;
    }
    im.mode = mode;
    const int nneed = mode == EF_JPEG_GRAY ? 1 : im.nc;  // grey output needs the luma plane only
    for (int k = 0; k < im.nc; ++k) {
      im.c[k].coef_off = B.coef_blocks * 64;
      B.coef_blocks += (int64_t)im.c[k].bw * im.c[k].bh;
      im.c[k].plane_off = B.plane_bytes;
      if (k < nneed) {
        B.plane_bytes += (int64_t)im.c[k].bw * 8 * im.c[k].bh * 8;
        B.block_start.push_back(B.blocks);
        B.ic.push_back((int)(B.imgs.size() << 2) | k);
        B.blocks += (int64_t)im.c[k].bw * im.c[k].bh;
      }
    }
    im.out_off = out_offsets ? out_offsets[i] : B.dense_out;
    B.dense_out += (int64_t)im.w * im.h * ch;
    B.px_start.push_back(B.pixels);
    B.pixels += (int64_t)im.w * im.h;
    B.img_of.push_back(i);
    B.imgs.push_back(im);
    B.data_bytes += sizes[i];
  }
}

}  // namespace
}  // namespace ef

using namespace ef;

extern "C" {

int ef_jpeg_info(const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count, int32_t* heights,
                 int32_t* widths, int32_t* components, int32_t* status) {
  if (count < 0 || (count > 0 && (!data || !offsets || !sizes))) return EF_E_INVALID;
  std::vector<HuffTab> pool;
  std::vector<unsigned short> qpool;
  std::vector<JSeg> segs;
  for (int i = 0; i < count; ++i) {
    JImage im{};
    pool.clear();
    qpool.clear();
    int st = sizes[i] > 0 ? parse(data + offsets[i], sizes[i], i, im, pool, qpool, segs, 0, false) : EF_JPEG_E_CORRUPT;
    if (st == 0 && (int64_t)im.w * im.h > ((int64_t)1 << 31)) st = EF_JPEG_E_UNSUPPORTED;
    if (heights) heights[i] = st == 0 ? im.h : 0;
    if (widths) widths[i] = st == 0 ? im.w : 0;
    if (components) components[i] = st == 0 ? im.nc : 0;
    if (status) status[i] = st;
  }
  return EF_OK;
}

int ef_jpeg_decode(ef_ctx* c, const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count,
                   int32_t mode, uint8_t* out, const int64_t* out_offsets, int32_t* status, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if (count < 0 || (count > 0 && (!data || !offsets || !sizes || !out || !out_offsets)) ||
      (mode != EF_JPEG_GRAY && mode != EF_JPEG_BGR))
    return set_err(c, EF_E_INVALID, "ef_jpeg_decode: bad arguments");
  if (count == 0) return EF_OK;
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  const bool dev_out = (flags & EF_MEM_DEVICE) != 0;
  const int ch = mode == EF_JPEG_GRAY ? 1 : 3;
  Batch B;
  build_batch(data, offsets, sizes, count, mode, dev_out ? out_offsets : nullptr, status, B);
  if (B.imgs.empty()) return EF_OK;
  // one pinned upload [files | images | Huffman tables | quant tables | segments | runs]
  // into the front of the device workspace; coefficients and sample planes follow
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  size_t off = 0;
  const size_t o_data = off; off += al((size_t)B.data_bytes + 16);
  const size_t o_imgs = off; off += al(B.imgs.size() * sizeof(JImage));
  const size_t o_pool = off; off += al(std::max<size_t>(B.pool.size(), 1) * sizeof(HuffTab));
  const size_t o_q = off; off += al(std::max<size_t>(B.qpool.size(), 1) * 2);
  const size_t o_seg = off; off += al(std::max<size_t>(B.segs.size(), 1) * sizeof(JSeg));
  const size_t o_bs = off; off += al(B.block_start.size() * 8);
  const size_t o_ic = off; off += al(B.ic.size() * 4);
  const size_t o_ps = off; off += al(B.px_start.size() * 8);
  const size_t up_bytes = off;
  const size_t o_coef = off; off += al((size_t)B.coef_blocks * 64 * 2);
  const size_t o_planes = off; off += al((size_t)B.plane_bytes + 16);
  // the previous call's upload may still be reading the pinned buffer
  {
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_err(c, e, "jpeg decode");
  }
  if (c->jpeg_pinned_bytes < up_bytes) {
    if (c->jpeg_pinned) (void)hipHostFree(c->jpeg_pinned);
    c->jpeg_pinned = nullptr;
    c->jpeg_pinned_bytes = 0;
    const hipError_t e = hipHostMalloc(&c->jpeg_pinned, up_bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
      c->jpeg_pinned = nullptr;
      return hip_err(c, e, "hipHostMalloc (jpeg staging)");
    }
    c->jpeg_pinned_bytes = up_bytes;
  }
  char* h = static_cast<char*>(c->jpeg_pinned);
  {
    int64_t o = 0;
    for (size_t i = 0; i < B.imgs.size(); ++i) {
      const int idx = B.img_of[i];
      std::memcpy(h + o_data + o, data + offsets[idx], (size_t)sizes[idx]);
      o += sizes[idx];
    }
    std::memset(h + o_data + o, 0, 16);
  }
  std::memcpy(h + o_imgs, B.imgs.data(), B.imgs.size() * sizeof(JImage));
  if (!B.pool.empty()) std::memcpy(h + o_pool, B.pool.data(), B.pool.size() * sizeof(HuffTab));
  if (!B.qpool.empty()) std::memcpy(h + o_q, B.qpool.data(), B.qpool.size() * 2);
  if (!B.segs.empty()) std::memcpy(h + o_seg, B.segs.data(), B.segs.size() * sizeof(JSeg));
  std::memcpy(h + o_bs, B.block_start.data(), B.block_start.size() * 8);
  std::memcpy(h + o_ic, B.ic.data(), B.ic.size() * 4);
  std::memcpy(h + o_ps, B.px_start.data(), B.px_start.size() * 8);
  {
    const int rc = ensure(c, c->jpeg_ws, off);
    if (rc != EF_OK) return rc;
  }
  uint8_t* dout = out;
  if (!dev_out) {
    const int rc = ensure(c, c->jpeg_out, (size_t)B.dense_out + 16);
    if (rc != EF_OK) return rc;
    dout = static_cast<uint8_t*>(c->jpeg_out.p);
  }
  char* base = static_cast<char*>(c->jpeg_ws.p);
  hipError_t e = hipMemcpyAsync(base, h, up_bytes, hipMemcpyHostToDevice, s);
  TimerEvt tev;
  timer_begin(c, EF_KERNEL_JPEG, &tev);
  if (e == hipSuccess) {
    const uint8_t* d_data = reinterpret_cast<const uint8_t*>(base + o_data);
    const JImage* d_imgs = reinterpret_cast<const JImage*>(base + o_imgs);
    short* d_coef = reinterpret_cast<short*>(base + o_coef);
    uint8_t* d_planes = reinterpret_cast<uint8_t*>(base + o_planes);
    if (!B.segs.empty())
      hipLaunchKernelGGL(jpeg_huff_kernel, dim3((unsigned)((B.segs.size() + 63) / 64)), dim3(64), 0, s, d_data,
                         reinterpret_cast<const JSeg*>(base + o_seg), (int)B.segs.size(), d_imgs,
                         reinterpret_cast<const HuffTab*>(base + o_pool), d_coef);
    if (B.blocks > 0)
      hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((B.blocks + kIdctBlocks - 1) / kIdctBlocks)), dim3(256), 0,
                         s, d_coef, d_imgs, reinterpret_cast<const int64_t*>(base + o_bs), (int)B.block_start.size(),
                         reinterpret_cast<const int*>(base + o_ic), reinterpret_cast<const unsigned short*>(base + o_q),
                         B.blocks, d_planes);
    if (B.pixels > 0)
      hipLaunchKernelGGL(jpeg_out_kernel, dim3((unsigned)((B.pixels + 255) / 256)), dim3(256), 0, s, d_imgs,
                         reinterpret_cast<const int64_t*>(base + o_ps), (int)B.imgs.size(), B.pixels, d_planes, dout);
    e = hipGetLastError();
  }
  timer_end(c, &tev);
  if (e != hipSuccess) return hip_err(c, e, "jpeg decode");
  if (dev_out) return EF_OK;  // stream-ordered, like the other EF_MEM_DEVICE calls
  std::vector<uint8_t> dense((size_t)B.dense_out);
  e = hipMemcpyAsync(dense.data(), dout, (size_t)B.dense_out, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_err(c, e, "jpeg decode");
  for (size_t i = 0; i < B.imgs.size(); ++i)
    std::memcpy(out + out_offsets[B.img_of[i]], dense.data() + B.imgs[i].out_off, (size_t)B.imgs[i].w * B.imgs[i].h * ch);
  return EF_OK;
}

int ef_jpeg_ingest(ef_ctx* c, const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count,
                   int32_t mode, int32_t out_h, int32_t out_w, uint8_t* out, int32_t* status, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if (count < 0 || out_h <= 0 || out_w <= 0 || (count > 0 && (!data || !offsets || !sizes || !out)) ||
      (mode != EF_JPEG_GRAY && mode != EF_JPEG_BGR))
    return set_err(c, EF_E_INVALID, "ef_jpeg_ingest: bad arguments");
  if (count == 0) return EF_OK;
  const int ch = mode == EF_JPEG_GRAY ? 1 : 3;
  const int64_t row = (int64_t)out_h * out_w;
  for (int32_t a = 0; a < count; a += 65535) {  // ef_preprocess's per-call image limit
    const int32_t m = std::min<int32_t>(65535, count - a);
    std::vector<int32_t> hh(m), ww(m), st(m), cc(m, ch);
    std::vector<int64_t> doff(m);
    int rc = ef_jpeg_info(data, offsets + a, sizes + a, m, hh.data(), ww.data(), nullptr, st.data());
    if (rc != EF_OK) return set_err(c, rc, "ef_jpeg_ingest: bad arguments");
    int64_t dense = 0;
    for (int32_t i = 0; i < m; ++i) {
      doff[i] = dense;
      if (st[i] == 0) dense += (int64_t)hh[i] * ww[i] * ch;
    }
    rc = ensure(c, c->jpeg_out, (size_t)dense + 256);
    if (rc != EF_OK) return rc;
    uint8_t* pix = static_cast<uint8_t*>(c->jpeg_out.p);
    rc = ef_jpeg_decode(c, data, offsets + a, sizes + a, m, mode, pix, doff.data(), st.data(), EF_MEM_DEVICE);
    if (rc != EF_OK) return rc;
    // a file the GPU decoder does not take becomes a 1x1 zero image: its row is zero
    bool any_bad = false;
    for (int32_t i = 0; i < m; ++i)
      if (st[i] != 0) {
        any_bad = true;
        doff[i] = dense;
        hh[i] = ww[i] = cc[i] = 1;
      }
    if (any_bad) {
      const hipError_t e = hipMemsetAsync(pix + dense, 0, 16, c->stream);
      if (e != hipSuccess) return hip_err(c, e, "jpeg ingest");
    }
    uint8_t* rows = out + (int64_t)a * row;
    if (!(flags & EF_MEM_DEVICE)) {  // host rows: resize into device staging, then copy out
      rc = ensure(c, c->jpeg_rows, (size_t)m * row);
      if (rc != EF_OK) return rc;
      rows = static_cast<uint8_t*>(c->jpeg_rows.p);
    }
    rc = ef_preprocess(c, pix, doff.data(), hh.data(), ww.data(), cc.data(), m, out_h, out_w, rows, EF_MEM_DEVICE);
    if (rc != EF_OK) return rc;
    if (!(flags & EF_MEM_DEVICE)) {
      hipError_t e = hipMemcpyAsync(out + (int64_t)a * row, rows, (size_t)m * row, hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) return hip_err(c, e, "jpeg ingest");
    }
    if (status) std::memcpy(status + a, st.data(), (size_t)m * 4);
  }
  return EF_OK;
}

}  // extern "C"

#ifdef EF_DIAGNOSTICS
// Diagnostic build only (never loaded by the package): the same per-thread device
// functions run in host loops, so decoder changes can be checked on a machine without
// a GPU (tools/micro/jpeg_host_check.py).  Output layout as ef_jpeg_decode's host form.
extern "C" int ef_diag_jpeg_decode_host(const uint8_t* data, const int64_t* offsets, const int64_t* sizes,
                                        int32_t count, int32_t mode, uint8_t* out, const int64_t* out_offsets,
                                        int32_t* status) {
  Batch B;
  build_batch(data, offsets, sizes, count, mode, out_offsets, status, B);
  std::vector<uint8_t> cat((size_t)B.data_bytes + 16, 0);
  int64_t o = 0;
  for (size_t i = 0; i < B.imgs.size(); ++i) {
    const int idx = B.img_of[i];
    std::memcpy(cat.data() + o, data + offsets[idx], (size_t)sizes[idx]);
    o += sizes[idx];
  }
  std::vector<short> coef((size_t)B.coef_blocks * 64 + 64);
  std::vector<uint8_t> planes((size_t)B.plane_bytes + 16);
  for (const JSeg& sg : B.segs) huff_segment(cat.data(), sg, B.imgs[sg.img], B.pool.data(), coef.data(), kNaturalHost);
  for (size_t r = 0; r < B.block_start.size(); ++r) {
    const JImage& im = B.imgs[B.ic[r] >> 2];
    const JComp& cp = im.c[B.ic[r] & 3];
    const unsigned short* q = B.qpool.data() + (int64_t)(im.qt_base + cp.q) * 64;
    for (int64_t b = 0; b < (int64_t)cp.bw * cp.bh; ++b) {
      int w[64];
      for (int j = 0; j < 8; ++j) idct_col(coef.data() + cp.coef_off + b * 64, q, j, w);
      const int by = (int)(b / cp.bw), bx = (int)(b % cp.bw);
      for (int j = 0; j < 8; ++j) {
        const unsigned long long v = idct_row(w, j);
        std::memcpy(planes.data() + cp.plane_off + ((int64_t)by * 8 + j) * cp.bw * 8 + (int64_t)bx * 8, &v, 8);
      }
    }
  }
  for (const JImage& im : B.imgs)
    for (int64_t k = 0; k < (int64_t)im.w * im.h; ++k) out_pixel(im, k, planes.data(), out);
  return EF_OK;
}
#endif
