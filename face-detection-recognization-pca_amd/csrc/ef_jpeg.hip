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
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ef_internal.hpp"
#include "ef_resize.hpp"

namespace ef {
namespace {

constexpr int kMaxComp = 3;

constexpr int kLookBits = 12;   // lookahead bits (libjpeg uses 8; 12 covers nearly every code)
constexpr int kLookSize = 1 << kLookBits;
constexpr int kLdsTables = 8;   // batches with at most this many distinct tables decode from LDS

struct HuffTab {                // libjpeg d_derived_tbl with a 12-bit lookahead
  unsigned short look[kLookSize];  // (nbits << 8) | symbol for codes <= 12 bits; nbits 0 = longer
  int maxcode[18];              // largest code of each length (-1: none), maxcode[17] sentinel
  int valoffset[18];            // huffval index offset per length
  unsigned char huffval[256];
};

struct JComp {
  int h, v;          // sampling factors
  int q;             // quantisation table index (Tables::quant)
  int dc, ac;        // Huffman table indices (Tables::huff)
  int bw, bh;        // blocks per row / column in the coefficient & sample planes
  int dw, dh;        // downsampled width / height (libjpeg's downsampled_width/height)
  int64_t coef_off;  // first block's int16[64] in the coefficient buffer
  int64_t plane_off; // first sample of the padded plane (bw * 8 bytes per row)
};

constexpr int kMaxBlocksPerMcu = 10;  // JPEG limit on blocks in one MCU (jdinput.c)

struct JImage {
  int w, h, nc, hmax, vmax;
  int mcux, mcuy;          // MCUs per row / column (interleaved), or blocks (one component)
  int interleaved;
  int restart;             // MCUs per restart interval (0 = none)
  int qt_base;             // 0: JComp::q indexes the batch's quantisation tables directly
  int bpm;                 // blocks per MCU
  unsigned char bcomp[kMaxBlocksPerMcu];  // component of each block of an MCU
  unsigned char boff[kMaxBlocksPerMcu];   // (row << 4) | column of that block inside the MCU
  JComp c[kMaxComp];
  int64_t out_off;
  int mode;                // EF_JPEG_GRAY / EF_JPEG_BGR
};

// An entropy segment: the whole scan, or one restart interval.  Its bytes are uploaded with
// the 0xFF00 stuffing removed (a clean big-endian bit string of nbits, zero beyond), and it
// is cut into chunks of chunk_bits for the parallel decode.
struct JSeg {
  int img;
  int mcu0, nmcu;     // first MCU and count
  int64_t beg, end;   // raw entropy-coded bytes [beg, end) inside the image's file
  int64_t word_off;   // first 32-bit word of the destuffed bits in the upload
  int nbits;
  int chunk0, nchunk;
};

// --------------------------------------------------------------------- host parsing
struct RawHuff {
  unsigned char bits[17];
  unsigned char val[256];
  bool present = false;
};

bool derive(const RawHuff& r, HuffTab& t, bool dc) {  // jdhuff.c jpeg_make_d_derived_tbl
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
  for (int i = 0; i < kLookSize; ++i) t.look[i] = 0;
  p = 0;
  for (int l = 1; l <= kLookBits; ++l)
    for (int i = 1; i <= r.bits[l]; ++i, ++p) {
      int lookbits = (int)code[p] << (kLookBits - l);
      for (int ctr = 1 << (kLookBits - l); ctr > 0; --ctr)
        t.look[lookbits++] = (unsigned short)((l << 8) | r.val[p]);
    }
  for (int i = 0; i < 256; ++i) t.huffval[i] = i < last ? r.val[i] : 0;
  if (dc)  // DC categories above 15 are rejected as libjpeg does (JERR_BAD_HUFF_TABLE)
    for (int i = 0; i < last; ++i)
      if (r.val[i] > 15) return false;
  return true;
}

// Derived Huffman and quantisation tables shared by the whole batch: files written by the
// same encoder carry identical tables, so the decode kernels see a handful of tables that
// stay resident in L1/L2 instead of one set per image.
struct Tables {
  std::vector<HuffTab> huff;
  std::vector<unsigned short> quant;  // 64 entries (natural order) per table
  std::unordered_map<std::string, int> huff_idx, quant_idx;
  std::vector<const std::string*> huff_key;  // key of each table in `huff` (for merging)
  // a table another Tables derived: index under its key, added if new
  int merge_huff(const std::string& key, const HuffTab& t) {
    auto it = huff_idx.find(key);
    if (it != huff_idx.end()) return it->second;
    const int idx = (int)huff.size();
    huff.push_back(t);
    huff_key.push_back(&huff_idx.emplace(key, idx).first->first);
    return idx;
  }
  int huff_table(const RawHuff& r, bool dc) {  // index, or -1 for an invalid table
    int cnt = 0;
    for (int l = 1; l <= 16; ++l) cnt += r.bits[l];
    std::string key(1, dc ? 'D' : 'A');
    key.append(reinterpret_cast<const char*>(r.bits + 1), 16);
    key.append(reinterpret_cast<const char*>(r.val), (size_t)std::min(cnt, 256));
    auto it = huff_idx.find(key);
    if (it != huff_idx.end()) return it->second;
    HuffTab t;
    const int idx = derive(r, t, dc) ? (int)huff.size() : -1;
    if (idx >= 0) huff.push_back(t);
    const std::string* kp = &huff_idx.emplace(std::move(key), idx).first->first;
    if (idx >= 0) huff_key.push_back(kp);
    return idx;
  }
  int quant_table(const unsigned short* q) {
    std::string key(reinterpret_cast<const char*>(q), 128);
    auto it = quant_idx.find(key);
    if (it != quant_idx.end()) return it->second;
    const int idx = (int)(quant.size() / 64);
    quant.insert(quant.end(), q, q + 64);
    quant_idx.emplace(std::move(key), idx);
    return idx;
  }
};

// Parse one file: frame, tables, scan, restart segments.  Returns 0 or a negative status.
int parse(const uint8_t* d, int64_t n, int img_index, JImage& im, Tables& T, std::vector<JSeg>& segs, bool want) {
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
        if (map_dc[td] < 0) map_dc[td] = T.huff_table(dht[0][td], true);
        if (map_ac[ta] < 0) map_ac[ta] = T.huff_table(dht[1][ta], false);
        if (map_dc[td] < 0 || map_ac[ta] < 0) return EF_JPEG_E_CORRUPT;
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
      im.qt_base = 0;
      for (int c = 0; c < im.nc; ++c) im.c[c].q = T.quant_table(qt[comp_q[c]]);
      // MCU block pattern (jdinput.c per_scan_setup, MCU_membership)
      im.bpm = 0;
      if (im.interleaved) {
        for (int c = 0; c < im.nc; ++c)
          for (int yy = 0; yy < im.c[c].v; ++yy)
            for (int xx = 0; xx < im.c[c].h; ++xx) {
              if (im.bpm >= kMaxBlocksPerMcu) return EF_JPEG_E_CORRUPT;
              im.bcomp[im.bpm] = (unsigned char)c;
              im.boff[im.bpm] = (unsigned char)((yy << 4) | xx);
              ++im.bpm;
            }
      } else {
        im.bpm = 1;
        im.bcomp[0] = 0;
        im.boff[0] = 0;
      }
      const int64_t total_mcu = (int64_t)im.mcux * im.mcuy;
      if (total_mcu * im.bpm > (int64_t)1 << 30) return EF_JPEG_E_UNSUPPORTED;
      if (!want) return 0;
      // entropy segments: the whole scan (the bit reader stops at the first marker), or
      // one per restart interval split at RSTn
      const int64_t scan_beg = p + 2 + len;
      if (n - scan_beg > ((int64_t)1 << 27)) return EF_JPEG_E_UNSUPPORTED;  // bit offsets stay in int32
      if (im.restart == 0) {
        segs.push_back(JSeg{img_index, 0, (int)total_mcu, scan_beg, n, 0, 0, 0, 0});
        return 0;
      }
      int64_t q = scan_beg, seg_beg = scan_beg;
      int mcu0 = 0;
      while (mcu0 < total_mcu) {
        bool rst = false;
        while (true) {  // next marker at or after q
          const void* f = q < n ? std::memchr(d + q, 0xFF, (size_t)(n - q)) : nullptr;
          if (!f) { q = n; break; }
          q = static_cast<const uint8_t*>(f) - d;
          if (q + 1 >= n) { q = n; break; }
          const int nx = d[q + 1];
          if (nx == 0x00) { q += 2; continue; }
          if (nx == 0xFF) { q += 1; continue; }
          rst = nx >= 0xD0 && nx <= 0xD7;
          break;
        }
        const int left = (int)(total_mcu - mcu0);
        if (rst) {
          const int cnt = std::min(im.restart, left);
          segs.push_back(JSeg{img_index, mcu0, cnt, seg_beg, q, 0, 0, 0, 0});
          mcu0 += cnt;
          q += 2;
          seg_beg = q;
          continue;
        }
        // EOI, another marker or the end of the data: the final interval.  A stream that
        // dropped RSTn markers relies on libjpeg's resynchronisation, which is not restated.
        if (left > im.restart) return EF_JPEG_E_UNSUPPORTED;
        segs.push_back(JSeg{img_index, mcu0, left, seg_beg, q, 0, 0, 0, 0});
        mcu0 += left;
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

// Destuffed big-endian bit string of one segment, read through 32-bit words into a 64-bit
// window; past the end it yields zeros, as libjpeg feeds zeros after a marker.  The words
// come from a queue refilled by one aligned 16-byte load per four words, issued a whole
// block ahead: the chunk loops are latency-bound (one dependent table lookup per symbol),
// and a word loaded only one refill ahead arrived too late (each lane streams its own chunk,
// so the loads do not coalesce).  The words array is 16-byte aligned and carries at least
// 32 bytes of readable slack past its last word (the block reads never fault; words past a
// segment's end read as zero).
struct BitStream {
  const unsigned* w;
  int nw;
  int pos;    // bit offset of the next unread bit
  int bits;   // valid bits in buf
  unsigned long long buf;
  unsigned q0, q1, q2, q3;  // the next words to append, q0 first (`left` of them valid)
  unsigned n0, n1, n2, n3;  // the aligned block after them (loaded ahead)
  int left;
  int wi;                   // segment word index of q0
  const unsigned* nb;       // the next aligned block to load
  __host__ __device__ unsigned word(int i) const { return i < nw ? __builtin_bswap32(w[i]) : 0u; }
  __host__ __device__ __forceinline__ void fetch() {
    n0 = nb[0];
    n1 = nb[1];
    n2 = nb[2];
    n3 = nb[3];
    nb += 4;
  }
  __host__ __device__ __forceinline__ void init(const unsigned* words, int nwords, int p) {
    w = words;
    nw = nwords;
    const int i = p >> 5, s = p & 31;
    buf = (unsigned long long)(word(i) << s) << 32;
    bits = 32 - s;
    pos = p;
    // queue from word i + 1: its aligned block, the words before it shifted out
    const unsigned* a = w + i + 1;
    const int off = (int)(((size_t)a >> 2) & 3);
    nb = a - off;
    fetch();
    q0 = n0, q1 = n1, q2 = n2, q3 = n3;
    for (int t = 0; t < off; ++t) q0 = q1, q1 = q2, q2 = q3;
    left = 4 - off;
    wi = i + 1;
    fetch();
  }
  __host__ __device__ __forceinline__ unsigned take() {
    const unsigned v = wi < nw ? __builtin_bswap32(q0) : 0u;
    ++wi;
    q0 = q1, q1 = q2, q2 = q3;
    if (--left == 0) {
      q0 = n0, q1 = n1, q2 = n2, q3 = n3;
      left = 4;
      fetch();
    }
    return v;
  }
  __host__ __device__ void refill() {  // afterwards at least 32 bits are buffered
    if (bits <= 32) {
      buf |= (unsigned long long)take() << (32 - bits);
      bits += 32;
    }
  }
  __host__ __device__ unsigned peek(int n) const { return (unsigned)(buf >> (64 - n)); }
  __host__ __device__ void skip(int n) {
    buf <<= n;
    bits -= n;
    pos += n;
  }
  __host__ __device__ int get(int n) {  // 1 <= n <= 16
    const int v = (int)peek(n);
    skip(n);
    return v;
  }
  // jdhuff.c HUFF_DECODE: lookahead table lut (t.look, or its copy in LDS), then the
  // canonical maxcode walk for longer codes
  __host__ __device__ int decode(const HuffTab& t, const unsigned short* lut) {
    const unsigned e = lut[peek(kLookBits)];
    if (e >> 8) {
      skip((int)(e >> 8));
      return (int)(e & 0xFF);
    }
    int l = kLookBits + 1;
    int code = (int)peek(l);
    while (l <= 16 && code > t.maxcode[l]) {
      ++l;
      code = (int)peek(l);
    }
    if (l > 16) {  // corrupt data: libjpeg warns, returns 0 having read 17 bits
      skip(17);
      return 0;
    }
    skip(l);
    return t.huffval[(code + t.valoffset[l]) & 0xFF];
  }
};

__host__ __device__ __forceinline__ int huff_extend(int x, int s) { return x < (1 << (s - 1)) ? x + (-1 << s) + 1 : x; }

// Decoder state at a codeword boundary: bit offset, block of the MCU, next coefficient
// index (0 = the block's DC symbol comes next).
__host__ __device__ __forceinline__ long long st_pack(int pos, int b, int k) {
  return ((long long)pos << 16) | (b << 8) | k;
}
__host__ __device__ __forceinline__ int st_pos(long long s) { return (int)(s >> 16); }
__host__ __device__ __forceinline__ int st_b(long long s) { return (int)((s >> 8) & 0xFF); }
__host__ __device__ __forceinline__ int st_k(long long s) { return (int)(s & 0xFF); }
constexpr long long kStateNone = -1;

// Per-image MCU description held in registers for the chunk loops (no global loads per
// symbol): the MCU layout packed 6 bits per block (comp | row << 2 | column << 4) into one
// 64-bit word read with a variable shift, and each component's tables and coefficient-plane
// geometry as named scalars.  (Arrays indexed by a run-time block or component number
// would be placed in scratch memory.)
constexpr int kMaxTables = 1 << 13;
struct McuInfo {
  unsigned long long layout;
  int bpm, mcux, interleaved;
  int dc0, dc1, dc2, ac0, ac1, ac2;
  int base0, base1, base2, bw0, bw1, bw2, h0, h1, h2, v0, v1, v2;
  __host__ __device__ __forceinline__ void load(const JImage& im) {
    bpm = im.bpm;
    mcux = im.mcux;
    interleaved = im.interleaved;
    layout = 0;
    for (int t = 0; t < im.bpm; ++t)
      layout |= (unsigned long long)(im.bcomp[t] | (im.boff[t] >> 4) << 2 | (im.boff[t] & 15) << 4) << (6 * t);
    dc0 = im.c[0].dc; ac0 = im.c[0].ac; base0 = (int)(im.c[0].coef_off / 64); bw0 = im.c[0].bw;
    h0 = im.c[0].h; v0 = im.c[0].v;
    dc1 = im.c[1].dc; ac1 = im.c[1].ac; base1 = (int)(im.c[1].coef_off / 64); bw1 = im.c[1].bw;
    h1 = im.c[1].h; v1 = im.c[1].v;
    dc2 = im.c[2].dc; ac2 = im.c[2].ac; base2 = (int)(im.c[2].coef_off / 64); bw2 = im.c[2].bw;
    h2 = im.c[2].h; v2 = im.c[2].v;
  }
  __host__ __device__ __forceinline__ unsigned info(int b) const { return (unsigned)(layout >> (6 * b)) & 63u; }
  __host__ __device__ static __forceinline__ int pick(int c, int a0, int a1, int a2) {
    return c == 0 ? a0 : (c == 1 ? a1 : a2);
  }
  // coefficient block of MCU block info bi in MCU (my, mx)
  __host__ __device__ __forceinline__ short* block(unsigned bi, int my, int mx, short* coef) const {
    const int c = bi & 3, yy = (bi >> 2) & 3, xx = (bi >> 4) & 3;
    const int by = interleaved ? my * pick(c, v0, v1, v2) + yy : my;
    const int bx = interleaved ? mx * pick(c, h0, h1, h2) + xx : mx;
    return coef + ((int64_t)pick(c, base0, base1, base2) + (int64_t)by * pick(c, bw0, bw1, bw2) + bx) * 64;
  }
};

struct CurTabs {  // the tables of the current MCU block
  const HuffTab* tdc;
  const HuffTab* tac;
  const unsigned short* ldc;
  const unsigned short* lac;
  int comp;
  __host__ __device__ __forceinline__ void set(const McuInfo& M, unsigned bi, const HuffTab* pool,
                                               const unsigned short* luts, int lstride) {
    comp = bi & 3;
    const int dc = McuInfo::pick(comp, M.dc0, M.dc1, M.dc2), ac = McuInfo::pick(comp, M.ac0, M.ac1, M.ac2);
    tdc = pool + dc;
    tac = pool + ac;
    ldc = luts + (int64_t)dc * lstride;
    lac = luts + (int64_t)ac * lstride;
  }
};

// Checkpoint of a chunk's decode trajectory: the state at the first codeword boundary at or
// past a fixed bit position, and the counts accumulated from the chunk start up to there.
struct Checkpoint {
  long long st;
  int n, d0, d1, d2, pad;
};
constexpr int kCheckpoints = 7;  // at 1/8 .. 7/8 of every chunk

// Synchronisation pass over one chunk: decode from state (b, k) at the stream's position to
// the first codeword boundary at or past end_bit, without storing coefficients.  Returns the
// exit state; cnt[0] = blocks started (DC symbols), cnt[1 + c] = sum of component c's DC
// differences.  With checkpoints (cp_bits > 0) the trajectory is recorded at start + m *
// cp_bits; when `merge` is set the recorded one is the chunk's previous trajectory, and the
// first checkpoint where the new decode lands in the same state ends the pass early: from
// there on both decodes are the same, so the exit is old_exit and the counts are the old
// ones shifted by the difference of the prefixes (the later checkpoints are shifted too).
__host__ __device__ __forceinline__ long long chunk_sync(const McuInfo& M, const HuffTab* pool, const unsigned short* luts,
                                         int lstride, BitStream& bs, int b, int k, int end_bit, int cnt[4],
                                         int start = 0, int cp_bits = 0, Checkpoint* cps = nullptr,
                                         bool merge = false, long long old_exit = 0) {
  int nblk = 0, dc0 = 0, dc1 = 0, dc2 = 0;
  int m = 1;
  int next_cp = cp_bits > 0 ? start + cp_bits : 0x7FFFFFFF;
  CurTabs T;
  T.set(M, M.info(b), pool, luts, lstride);
  while (bs.pos < end_bit) {
    while (bs.pos >= next_cp) {  // (one step can pass several checkpoints)
      const long long st = st_pack(bs.pos, b, k);
      Checkpoint& c = cps[m - 1];
      if (merge && st == c.st) {
#if defined(EF_DIAGNOSTICS) && !defined(__HIP_DEVICE_COMPILE__)
        if (std::getenv("EF_JPEG_CHECK")) {
          BitStream b2 = bs;
          int c4[4];
          const long long e2 = chunk_sync(M, pool, luts, lstride, b2, b, k, end_bit, c4);
          if (e2 != old_exit)
            std::fprintf(stderr, "bad merge at cp %d pos %d: continuation exit %lld, old exit %lld\n", m, bs.pos, e2,
                         old_exit);
        }
#endif
        const int dn = nblk - c.n, e0 = dc0 - c.d0, e1 = dc1 - c.d1, e2 = dc2 - c.d2;
        for (int q = m - 1; q < kCheckpoints; ++q) {
          cps[q].n += dn;
          cps[q].d0 += e0;
          cps[q].d1 += e1;
          cps[q].d2 += e2;
        }
        cnt[0] += dn;
        cnt[1] += e0;
        cnt[2] += e1;
        cnt[3] += e2;
        return old_exit;
      }
      c.st = st;
      c.n = nblk;
      c.d0 = dc0;
      c.d1 = dc1;
      c.d2 = dc2;
      next_cp = ++m <= kCheckpoints ? start + m * cp_bits : 0x7FFFFFFF;
    }
    bs.refill();
    // one symbol decode for DC and AC alike (the table is selected, not the code path): the
    // lanes of a wave sit at DC and AC symbols at once, and two decode paths would serialise
    // two table lookups per step
    const bool dc = k == 0;
    const int sym = bs.decode(dc ? *T.tdc : *T.tac, dc ? T.ldc : T.lac);
    const int s = dc ? sym : (sym & 15), r = dc ? 0 : (sym >> 4);
    const int bitsv = s ? bs.get(s) : 0;
    if (dc) {
      const int diff = s ? huff_extend(bitsv, s) : 0;
      dc0 += T.comp == 0 ? diff : 0;
      dc1 += T.comp == 1 ? diff : 0;
      dc2 += T.comp == 2 ? diff : 0;
      ++nblk;
      k = 1;
    } else if (s) {
      k += r + 1;
    } else {
      k = r == 15 ? k + 16 : 64;
    }
    if (k >= 64) {
      k = 0;
      b = b + 1 == M.bpm ? 0 : b + 1;
      T.set(M, M.info(b), pool, luts, lstride);
    }
  }
  const long long exit_st = st_pack(bs.pos, b, k);
  for (; m <= kCheckpoints && next_cp != 0x7FFFFFFF; ++m) {  // checkpoints the last step jumped past
    Checkpoint& c = cps[m - 1];
    c.st = exit_st;
    c.n = nblk;
    c.d0 = dc0;
    c.d1 = dc1;
    c.d2 = dc2;
  }
  cnt[0] = nblk;
  cnt[1] = dc0;
  cnt[2] = dc1;
  cnt[3] = dc2;
  return exit_st;
}

// Output pass over one chunk from its exact start state: g = index (in the segment) of the
// next block to start, pred = DC predictors there.  Stops at the first codeword boundary at
// or past end_bit, or once all `total` blocks of the segment are decoded.  Coefficients are
// stored straight into the zeroed coefficient buffer (a block shared with a neighbouring
// chunk gets disjoint coefficients from each).  Measured against assembling each block in
// LDS and writing it as one 128-byte piece, the direct stores were faster: the per-block
// flush runs divergently in nearly every step of a 64-chunk wave.
__host__ __device__ __forceinline__ void chunk_write(const McuInfo& M, int mcu0, const HuffTab* pool,
                                                     const unsigned short* luts, int lstride, BitStream& bs, int b,
                                                     int k, int end_bit, int g, int total, int pred[3], short* coef,
                                                     const unsigned char* nat) {
  if (k > 0 && g == 0) return;  // inconsistent state (cannot happen for an exact state)
  int mcu = mcu0 + (k > 0 ? g - 1 : g) / M.bpm;
  int my = mcu / M.mcux, mx = mcu - my * M.mcux;
  unsigned bi = M.info(b);
  CurTabs T;
  T.set(M, bi, pool, luts, lstride);
  short* blk = k > 0 ? M.block(bi, my, mx, coef) : nullptr;
  while (bs.pos < end_bit) {
    if (k == 0 && g >= total) break;
    bs.refill();
    // one symbol decode and one store path for DC and AC alike (see chunk_sync)
    const bool dc = k == 0;
    if (dc) {
      blk = M.block(bi, my, mx, coef);
      ++g;
    }
    const int sym = bs.decode(dc ? *T.tdc : *T.tac, dc ? T.ldc : T.lac);
    const int s = dc ? sym : (sym & 15), r = dc ? 0 : (sym >> 4);
    const int val = s ? huff_extend(bs.get(s), s) : 0;
    int v = val, pos = 0;
    if (dc) {
      if (T.comp == 0) v = pred[0] += val;
      else if (T.comp == 1) v = pred[1] += val;
      else v = pred[2] += val;
      k = 1;
    } else if (s) {
      k += r;
      pos = nat[k];
      ++k;
    } else {
      k = r == 15 ? k + 16 : 64;
    }
    if (dc || s) blk[pos] = (short)v;
    if (k >= 64) {
      k = 0;
      if (++b == M.bpm) {
        b = 0;
        if (++mx == M.mcux) {
          mx = 0;
          ++my;
        }
      }
      bi = M.info(b);
      T.set(M, bi, pool, luts, lstride);
    }
  }
}

struct ChunkCtx {  // what the chunk kernels share
  const int* chunk_seg;
  const JSeg* segs;
  const JImage* imgs;
  const HuffTab* pool;
  const unsigned* words;
  int nchunks;
  int chunk_bits;
  int warm_bits;  // round-0 warm-up before each chunk (<= chunk_bits)
  Checkpoint* cps;  // kCheckpoints per chunk
};

__host__ __device__ __forceinline__ void chunk_stream(const ChunkCtx& X, const JSeg& sg, int pos, BitStream& bs) {
  bs.init(X.words + sg.word_off, (sg.nbits + 31) >> 5, pos);
}

// One synchronisation round (Weissenberger & Schmidt's self-synchronising parallel Huffman
// decoding, with the JPEG syntax position in the state).  Round 0: every chunk decodes from
// a guess — block 0, DC next, warm_bits before its first bit — and takes the state at its
// first codeword boundary as its start, except a segment's first chunk, whose start is
// exact.  Round t: chunk i adopts chunk i-1's exit state of round t-1 when it differs
// from the one it started from, re-decodes and raises *changed.  At the fixed point every
// start state is exact by induction from the segment start.  Last chunks of a segment only
// record their start state (nothing follows them).
__host__ __device__ __forceinline__ void sync_chunk(const ChunkCtx& X, const HuffTab* pool, const unsigned short* luts,
                                                    int lstride, int i, int round,
                                    long long* S, const long long* Ein, long long* Eout, int* cnt, int* changed) {
  const JSeg& sg = X.segs[X.chunk_seg[i]];
  const int j = i - sg.chunk0;
  const bool last = j == sg.nchunk - 1;
  long long s;
  if (round == 0) {
    s = st_pack(j * X.chunk_bits, 0, 0);
    S[i] = s;
  } else {
    if (j == 0) {
      Eout[i] = Ein[i];
      return;
    }
    s = Ein[i - 1];
    if (s == S[i]) {
      Eout[i] = Ein[i];
      return;
    }
    S[i] = s;
  }
  if (last) {
    Eout[i] = kStateNone;
    return;
  }
  McuInfo M;
  M.load(X.imgs[sg.img]);
  BitStream bs;
  const int start = j * X.chunk_bits, end = (j + 1) * X.chunk_bits;
  const int cp_bits = X.chunk_bits / (kCheckpoints + 1);
  Checkpoint* cps = X.cps + (int64_t)i * kCheckpoints;
  if (round == 0) {
    if (j > 0) {
      // warm-up: decode from a guess X.warm_bits before the chunk; the state at its first
      // codeword boundary is often already exact
      chunk_stream(X, sg, start - X.warm_bits, bs);
      int dummy[4];
      // (cps passed although no checkpoint is taken here: a null pointer merged with the
      // global one would make the checkpoint stores flat)
      s = chunk_sync(M, pool, luts, lstride, bs, 0, 0, start, dummy, 0, 0, cps);
      S[i] = s;
    } else {
      chunk_stream(X, sg, st_pos(s), bs);
    }
    Eout[i] = chunk_sync(M, pool, luts, lstride, bs, st_b(s), st_k(s), end, cnt + 4 * i, start, cp_bits, cps);
    return;
  }
  chunk_stream(X, sg, st_pos(s), bs);
  const long long e = chunk_sync(M, pool, luts, lstride, bs, st_b(s), st_k(s), end, cnt + 4 * i, start, cp_bits,
                                 cps, true, Ein[i]);
  Eout[i] = e;
  if (e != Ein[i]) *changed = 1;  // only a changed exit can change the next chunk
}

constexpr int kChunkThreads = 256;
constexpr int kDeviceRounds = 8;  // synchronisation rounds queued without a host round trip
constexpr int kGlobalLutStride = (int)(sizeof(HuffTab) / 2);

// The batch's Huffman tables (lookahead table, maxcode / valoffset / huffval for codes longer
// than the lookahead) copied whole into LDS when there are at most kLdsTables of them (the
// usual case: one encoder's 4 tables), else read from the global pool.  The chunk loops are
// instantiated once per case, so the LDS case's table pointer is known to point into LDS
// and every lookup is a ds_read: a pointer that may point to either memory is a flat access,
// whose wait also drains every outstanding global load and store — the bit stream's prefetch
// and the coefficient stores — at each symbol.  The long-code tables must be in LDS too:
// codes over 12 bits are rare, but a 64-lane wave meets one in most steps, and their
// dependent maxcode reads from global memory then stall the whole wave.
constexpr int kTabBytes = (int)sizeof(HuffTab);
template <class F>
__device__ __forceinline__ void with_luts(const ChunkCtx& X, int lds_tables, unsigned short* smem, const F& f) {
  if (lds_tables == 0) {
    f(X.pool, X.pool[0].look, kGlobalLutStride);
    return;
  }
  const int nvec = lds_tables * (kTabBytes / 16);
  for (int t = threadIdx.x; t < nvec; t += blockDim.x)
    reinterpret_cast<uint4*>(smem)[t] = reinterpret_cast<const uint4*>(X.pool)[t];
  __syncthreads();
  const HuffTab* lp = reinterpret_cast<const HuffTab*>(smem);
  f(lp, lp[0].look, kGlobalLutStride);
}

// prev_changed (rounds >= 2 of the device-side sequence): the previous round's change flag;
// when it stayed 0 the fixed point is reached and this round — and, its own flag staying
// 0, every later one — exits at once, so rounds can be queued without a host round trip.
__global__ __launch_bounds__(kChunkThreads) void jpeg_sync_kernel(ChunkCtx X, int lds_tables, int round,
                                                                  long long* __restrict__ S,
                                                                  const long long* __restrict__ Ein,
                                                                  long long* __restrict__ Eout, int* __restrict__ cnt,
                                                                  int* __restrict__ changed,
                                                                  const int* __restrict__ prev_changed) {
  if (prev_changed && *prev_changed == 0) return;  // uniform: converged before this round
  extern __shared__ unsigned short slut[];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  with_luts(X, lds_tables, slut, [&](const HuffTab* pool, const unsigned short* luts, int lstride) {
    if (i < X.nchunks) sync_chunk(X, pool, luts, lstride, i, round, S, Ein, Eout, cnt, changed);
  });
}

// Completion of one segment after r synchronisation rounds, sequentially along its chunks.
// After round r chunks 0..r start exactly (induction from the segment start), and after
// every round E[i] is the exit of a decode from S[i] (cnt[i] its counts).  So walking
// j = r+1, r+2, …: E[i-1] is exact; when it equals S[i] chunk i is already exact, else
// chunk i re-decodes from it (merging into its old trajectory at the first shared
// checkpoint, as a round does).  Replaces further rounds for the rare batch whose rounds
// have not reached the fixed point after the queued ones — without a host round trip.
__host__ __device__ __forceinline__ void finish_segment(const ChunkCtx& X, const unsigned short* luts, int lstride,
                                                        const JSeg& sg, int r, long long* S, long long* E, int* cnt) {
  if (sg.nchunk <= r + 1) return;
  McuInfo M;
  M.load(X.imgs[sg.img]);
  const int cp_bits = X.chunk_bits / (kCheckpoints + 1);
  for (int j = r + 1; j < sg.nchunk; ++j) {
    const int i = sg.chunk0 + j;
    const long long s = E[i - 1];
    if (s == S[i]) continue;
    S[i] = s;
    if (j == sg.nchunk - 1) {
      E[i] = kStateNone;
      break;
    }
    BitStream bs;
    chunk_stream(X, sg, st_pos(s), bs);
    E[i] = chunk_sync(M, X.pool, luts, lstride, bs, st_b(s), st_k(s), (j + 1) * X.chunk_bits, cnt + 4 * i,
                      j * X.chunk_bits, cp_bits, X.cps + (int64_t)i * kCheckpoints, true, E[i]);
  }
}

// One thread per segment; returns at once when the last queued round changed nothing.
__global__ __launch_bounds__(64) void jpeg_finish_kernel(ChunkCtx X, int nseg, int r, long long* __restrict__ S,
                                                         long long* __restrict__ E, int* __restrict__ cnt,
                                                         const int* __restrict__ last_changed) {
  if (*last_changed == 0) return;
  const int si = blockIdx.x * blockDim.x + threadIdx.x;
  if (si < nseg) finish_segment(X, X.pool[0].look, kGlobalLutStride, X.segs[si], r, S, E, cnt);
}

// Exclusive scan of the chunk counts inside each segment: first block index and DC
// predictors at every chunk's start.
__host__ __device__ __forceinline__ void scan_segment(const ChunkCtx& X, const JSeg& sg, const int* cnt, int* G, int* P) {
  int g = 0, p0 = 0, p1 = 0, p2 = 0;
  for (int j = 0; j < sg.nchunk; ++j) {
    const int i = sg.chunk0 + j;
    G[i] = g;
    P[3 * i] = p0;
    P[3 * i + 1] = p1;
    P[3 * i + 2] = p2;
    if (j + 1 < sg.nchunk) {
      g += cnt[4 * i];
      p0 += cnt[4 * i + 1];
      p1 += cnt[4 * i + 2];
      p2 += cnt[4 * i + 3];
    }
  }
}

__global__ __launch_bounds__(64) void jpeg_scan_kernel(ChunkCtx X, int nseg, const int* __restrict__ cnt,
                                                      int* __restrict__ G, int* __restrict__ P) {
  const int si = blockIdx.x * blockDim.x + threadIdx.x;
  if (si < nseg) scan_segment(X, X.segs[si], cnt, G, P);
}

__host__ __device__ __forceinline__ void write_chunk(const ChunkCtx& X, const HuffTab* pool, const unsigned short* luts,
                                                     int lstride, int i,
                                                     const long long* S, const int* G, const int* P, short* coef,
                                                     const unsigned char* nat) {
  const JSeg& sg = X.segs[X.chunk_seg[i]];
  const int j = i - sg.chunk0;
  const long long s = S[i];
  BitStream bs;
  chunk_stream(X, sg, st_pos(s), bs);
  int pred[3] = {P[3 * i], P[3 * i + 1], P[3 * i + 2]};
  const int end = j == sg.nchunk - 1 ? 0x7FFFFFFF : (j + 1) * X.chunk_bits;
  McuInfo M;
  M.load(X.imgs[sg.img]);
  chunk_write(M, sg.mcu0, pool, luts, lstride, bs, st_b(s), st_k(s), end, G[i], sg.nmcu * M.bpm, pred, coef, nat);
}

// LDS: [Huffman tables | natural order]
__global__ __launch_bounds__(kChunkThreads) void jpeg_write_kernel(ChunkCtx X, int lds_tables,
                                                                   const long long* __restrict__ S,
                                                                   const int* __restrict__ G, const int* __restrict__ P,
                                                                   short* __restrict__ coef) {
  extern __shared__ unsigned short slut[];
  unsigned char* snat = reinterpret_cast<unsigned char*>(slut) + lds_tables * kTabBytes;
  if (threadIdx.x < 80) snat[threadIdx.x] = kNatural[threadIdx.x];
  if (lds_tables == 0) __syncthreads();  // (with_luts' staging ends with one otherwise)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  with_luts(X, lds_tables, slut, [&](const HuffTab* pool, const unsigned short* luts, int lstride) {
    if (i < X.nchunks) write_chunk(X, pool, luts, lstride, i, S, G, P, coef, snat);
  });
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
  const int64_t gb0 = (int64_t)blockIdx.x * kIdctBlocks, gb = gb0 + lb;
  if (gb >= total_blocks) return;  // whole 8-lane groups leave together
  int lo = 0, hi = nruns - 1;  // the (image, component) run holding the workgroup's first block
  while (lo < hi) {  // (uniform: scalar loads)
    const int mid = (lo + hi + 1) >> 1;
    if (block_start[mid] <= gb0) lo = mid; else hi = mid - 1;
  }
  while (lo + 1 < nruns && block_start[lo + 1] <= gb) ++lo;  // then this group's run
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
__host__ __device__ void out_pixel(const JImage& im, int y, int x, const uint8_t* planes, uint8_t* out) {
  const int64_t k = (int64_t)y * im.w + x;
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

// One wave per output row (the image found once per wave from the row starts), lanes
// stride across the row.
__host__ __device__ __forceinline__ unsigned load4(const uint8_t* p) {  // 4-byte aligned
  return *reinterpret_cast<const unsigned*>(p);
}

// Fancy-upsampled chroma of output columns x0..x0+3 (x0 % 4 == 0) of row y for a component
// subsampled 2x horizontally (v2: and vertically) with downsampled_width > 2: the same
// jdsample.c arithmetic as upsample(), sharing the column sums of chroma columns
// j0-1 .. j0+2 between the four pixels.
__host__ __device__ __forceinline__ void upsample_h2_quad(const uint8_t* pl, const JComp& cp, bool v2, int y, int x0,
                                                          int o[4]) {
  const int64_t pitch = (int64_t)cp.bw * 8;
  const int j0 = x0 >> 1, last = cp.dw - 1, wmax = cp.bw * 8 - 1;
  const uint8_t* r0 = pl + (int64_t)(v2 ? y >> 1 : y) * pitch;
  const uint8_t* r1 = r0;
  if (v2) {
    int i1 = (y & 1) ? (y >> 1) + 1 : (y >> 1) - 1;
    i1 = i1 < 0 ? 0 : (i1 > cp.dh - 1 ? cp.dh - 1 : i1);
    r1 = pl + (int64_t)i1 * pitch;
  }
  int cs[4];  // column sums of chroma columns j0-1 .. j0+2 (clamped into the padded row)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    int c = j0 - 1 + t;
    c = c < 0 ? 0 : (c > wmax ? wmax : c);
    cs[t] = v2 ? r0[c] * 3 + r1[c] : r0[c];
  }
  // h2v2: 3 * nearer + further, rounding 8 / 7 >> 4;  h2v1: 3 * nearer + further, 1 / 2 >> 2
  const int sh = v2 ? 4 : 2, b0 = v2 ? 8 : 1, b1 = v2 ? 7 : 2;
#pragma unroll
  for (int p = 0; p < 2; ++p) {  // chroma column j = j0 + p -> output columns 2j, 2j+1
    const int j = j0 + p;
    const int c = cs[p + 1];
    o[2 * p] = j == 0 ? (v2 ? (c * 4 + 8) >> 4 : c) : (c * 3 + cs[p] + b0) >> sh;
    o[2 * p + 1] = j == last ? (v2 ? (c * 4 + 7) >> 4 : c) : (c * 3 + cs[p + 2] + b1) >> sh;
  }
}

// Output columns x0..x0+3 of row y (those < w): one Y word, shared chroma column sums; the
// general per-pixel path covers grey sources, box upsampling and the rest.
__host__ __device__ __forceinline__ void out_quad(const JImage& im, int y, int x0, const uint8_t* planes,
                                                  uint8_t* out) {
  const int n = im.w - x0 < 4 ? im.w - x0 : 4;
  const uint8_t* prow = planes + im.c[0].plane_off + (int64_t)y * im.c[0].bw * 8;
  if (im.mode == EF_JPEG_GRAY) {
    for (int t = 0; t < n; ++t) out[im.out_off + (int64_t)y * im.w + x0 + t] = prow[x0 + t];
    return;
  }
  const JComp& cb = im.c[1];
  const JComp& cr = im.c[2];
  const bool h2 = im.nc == 3 && im.hmax == 2 * cb.h && cb.h == cr.h && cb.v == cr.v && cb.dw > 2;
  const bool full = im.nc == 3 && im.hmax == cb.h && im.vmax == cb.v && cb.h == cr.h && cb.v == cr.v;
  if (!h2 && !full) {
    for (int t = 0; t < n; ++t) out_pixel(im, y, x0 + t, planes, out);
    return;
  }
  const unsigned yw = load4(prow + x0);
  int ub[4], vr[4];
  if (h2) {
    const bool v2 = im.vmax == 2 * cb.v;
    upsample_h2_quad(planes + cb.plane_off, cb, v2, y, x0, ub);
    upsample_h2_quad(planes + cr.plane_off, cr, v2, y, x0, vr);
  } else {
    const unsigned bw = load4(planes + cb.plane_off + (int64_t)y * cb.bw * 8 + x0);
    const unsigned rw = load4(planes + cr.plane_off + (int64_t)y * cr.bw * 8 + x0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      ub[t] = (bw >> (8 * t)) & 255;
      vr[t] = (rw >> (8 * t)) & 255;
    }
  }
  uint8_t* o = out + im.out_off + 3 * ((int64_t)y * im.w + x0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < n) {
      const int Y = (yw >> (8 * t)) & 255;
      o[3 * t] = clamp255(Y + cb_b(ub[t]));
      o[3 * t + 1] = clamp255(Y + cbcr_g(ub[t], vr[t]));
      o[3 * t + 2] = clamp255(Y + cr_r(vr[t]));
    }
  }
}

// One wave per output row (the image found once per wave from the row starts), each lane
// four adjacent pixels.
__global__ __launch_bounds__(256) void jpeg_out_kernel(const JImage* __restrict__ imgs, const int64_t* __restrict__ row_start,
                                                      int nimg, int64_t total_rows, const uint8_t* __restrict__ planes,
                                                      uint8_t* __restrict__ out) {
  const int64_t r = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (r >= total_rows) return;
  int lo = 0, hi = nimg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (row_start[mid] <= r) lo = mid; else hi = mid - 1;
  }
  const JImage& im = imgs[lo];
  const int y = (int)(r - row_start[lo]);
  for (int x0 = 4 * (threadIdx.x & 63); x0 < im.w; x0 += 256) out_quad(im, y, x0, planes, out);
}

// Source rows output row dy of an (oh x ow) resize of an (h x w) image reads (resize_px's
// three cases): first and last.
__device__ __forceinline__ void resize_rows(int h, int w, int oh, int ow, int dy, int& r0, int& r1) {
  if (oh == h && ow == w) {
    r0 = r1 = dy;
  } else if (h == 2 * oh && w == 2 * ow) {
    r0 = 2 * dy;
    r1 = 2 * dy + 1;
  } else {
    int a, b;
    lin_axis(dy, h, oh, false, r0, r1, a, b);
  }
}

// Chroma rows of component cp that luma rows [ya, yb] read through upsample().
__device__ __forceinline__ void chroma_rows(const JComp& cp, int vmax, int ya, int yb, int& ca, int& cb) {
  if (vmax == 2 * cp.v) {
    ca = max((ya >> 1) - 1, 0);
    cb = min((yb >> 1) + 1, cp.dh - 1);
  } else {
    ca = ya;
    cb = yb;
  }
}

// Ingest: rows [kResizeBand * blockIdx.x, +kResizeBand) of file blockIdx.y's (oh x ow) grey
// output (ef_preprocess's arithmetic) straight from the decoded planes, without writing the
// full-size BGR image and reading it back.  The band's luma rows and the chroma rows their
// upsampling reads are first copied into LDS with coalesced dword loads (each output pixel
// otherwise gathers ~36 single bytes: 4 samples x (Y + 2 x 4 chroma)); the samples are then
// formed from LDS by the same functions (pointers into LDS offset by the first staged row).
// A band whose rows exceed the LDS budget (very wide sources) reads the planes directly.
// The budget is kept small so that 8 blocks fit per CU: the kernel is latency-bound (three
// dependent loads — file map, image record, rows — before a block computes), and a 40 KiB
// budget (4 blocks per CU) measured no faster than the gathers it replaced (0.43 ms).
// file_img[f] < 0 (a file the decoder does not take) gives a zero row, as the resize of a
// 1x1 zero image does.
constexpr int kResizeBand = 4;          // output rows per block (256 threads: one pixel each at 64 wide)
constexpr int kResizeLds = 16 * 1024;   // 8 blocks of 4 waves per CU (a 325-px 4:2:0 source needs ~11 KiB)
__global__ __launch_bounds__(256) void jpeg_resize_kernel(const JImage* __restrict__ imgs, const int* __restrict__ file_img,
                                                         const uint8_t* __restrict__ planes, int oh, int ow,
                                                         uint8_t* __restrict__ dst) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kResizeLds / 4];
  const int dy0 = blockIdx.x * kResizeBand, dy1 = min(dy0 + kResizeBand, oh);
  uint8_t* rows = dst + (int64_t)blockIdx.y * oh * ow;
  const int ii = file_img[blockIdx.y];
  const int nout = (dy1 - dy0) * ow;
  if (ii < 0) {
    for (int o = threadIdx.x; o < nout; o += 256) rows[dy0 * ow + o] = 0;
    return;
  }
  const JImage& im = imgs[ii];
  const bool colour = !(im.mode == EF_JPEG_GRAY || im.nc == 1);
  int ya, yb, t;
  resize_rows(im.h, im.w, oh, ow, dy0, ya, t);
  resize_rows(im.h, im.w, oh, ow, dy1 - 1, t, yb);
  const int64_t py = (int64_t)im.c[0].bw * 8;
  int c1a = 0, c1b = -1, c2a = 0, c2b = -1;
  int64_t p1 = 0, p2 = 0;
  if (colour) {
    chroma_rows(im.c[1], im.vmax, ya, yb, c1a, c1b);
    chroma_rows(im.c[2], im.vmax, ya, yb, c2a, c2b);
    p1 = (int64_t)im.c[1].bw * 8;
    p2 = (int64_t)im.c[2].bw * 8;
  }
  const int64_t ny = (yb - ya + 1) * py, n1 = (c1b - c1a + 1) * p1, n2 = (c2b - c2a + 1) * p2;
  const uint8_t* Yp = planes + im.c[0].plane_off;
  const uint8_t* Cb = planes + im.c[1].plane_off;
  const uint8_t* Cr = planes + im.c[2].plane_off;
  const auto run = [&](const uint8_t* Yq, const uint8_t* Cbq, const uint8_t* Crq) {
    const auto gray = [&](int y, int x) {
      const int Y = Yq[(int64_t)y * py + x];
      if (!colour) return Y;
      const int cb = upsample(Cbq, im.c[1], im.hmax, im.vmax, y, x);
      const int cr = upsample(Crq, im.c[2], im.hmax, im.vmax, y, x);
      const int b = clamp255(Y + cb_b(cb)), g = clamp255(Y + cbcr_g(cb, cr)), r = clamp255(Y + cr_r(cr));
      return (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14;
    };
    for (int o = threadIdx.x; o < nout; o += 256) {
      const int dy = dy0 + o / ow, dx = o - (o / ow) * ow;
      rows[dy * ow + dx] = (uint8_t)resize_px(gray, im.h, im.w, oh, ow, dy, dx);
    }
  };
  if (ny + n1 + n2 > kResizeLds) {  // uniform: a band too wide for LDS reads the planes directly
    run(Yp, Cb, Cr);
    return;
  }
  // stage the band's rows (pitches are multiples of 8, planes 64-byte aligned)
  const auto stage = [&](const uint8_t* src, int64_t bytes, int64_t at) {
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
    for (int64_t e = threadIdx.x; e < bytes / 4; e += 256) lds[at / 4 + e] = s4[e];
  };
  stage(Yp + ya * py, ny, 0);
  if (colour) {
    stage(Cb + c1a * p1, n1, ny);
    stage(Cr + c2a * p2, n2, ny + n1);
  }
  __syncthreads();
  // row r of a plane at (r - its first staged row) * pitch in LDS
  const uint8_t* l8 = reinterpret_cast<const uint8_t*>(lds);
  run(l8 - ya * py, l8 + ny - c1a * p1, l8 + ny + n1 - c2a * p2);
}

// Diagnostic build: wall time of the host stages of a decode (EF_JPEG_TIMES=1 prints them).
#ifdef EF_DIAGNOSTICS
struct StageTimer {
  const bool on = std::getenv("EF_JPEG_TIMES") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what, hipStream_t s = nullptr, bool sync = false) {
    if (!on) return;
    if (sync) (void)hipStreamSynchronize(s);
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[jpeg] %-12s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};
#else
struct StageTimer {
  void mark(const char*, hipStream_t = nullptr, bool = false) {}
};
#endif

// ------------------------------------------------------------------ batch layout
// Everything one decode launch needs, built on the host: per-image geometry, Huffman and
// quantisation tables, entropy segments and their chunks, IDCT runs, output pixel starts.
struct Batch {
  Tables T;
  std::vector<JSeg> segs;
  std::vector<JImage> imgs;
  std::vector<int> img_of;            // input index of each decoded image
  std::vector<int64_t> block_start;   // IDCT runs: first global block of (image, component)
  std::vector<int> ic;                // (image << 2) | component of each run
  std::vector<int64_t> row_start;     // first output row of each image (rows of all images in order)
  std::vector<int> chunk_seg;         // segment of each chunk
  std::vector<int> file_img;          // ingest: image of each input file of the batch (-1: not decoded here)
  int64_t words = 0;                  // 32-bit words reserved for the destuffed segments
  int chunk_bits = 0, warm_bits = 0;
  int64_t coef_blocks = 0, plane_bytes = 0, blocks = 0, rows = 0, dense_out = 0;
};

// out_offsets: images land there (device layout); null: packed densely.
// The per-file marker parse runs on host threads (one Tables and segment list per thread),
// merged in file order afterwards: the same images, segments and layout as a sequential
// parse, with the batch tables deduplicated in the order the accepted files use them.
void build_batch(const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int count, int mode,
                 const int64_t* out_offsets, int32_t* status, Batch& B) {
  const int ch = mode == EF_JPEG_GRAY ? 1 : 3;
  struct FileRes {
    JImage im;
    int st = 0, seg_beg = 0, seg_end = 0;
  };
  std::vector<FileRes> R((size_t)std::max(count, 0));
  const int nt = count >= 512 ? host_threads() : 1;
  std::vector<Tables> TT(nt);
  std::vector<std::vector<JSeg>> SS(nt);
  auto work = [&](int t, int a, int e) {
    for (int i = a; i < e; ++i) {
      FileRes& f = R[i];
      f.im = JImage{};
      f.seg_beg = (int)SS[t].size();
      f.st = sizes[i] > 0 ? parse(data + offsets[i], sizes[i], i, f.im, TT[t], SS[t], true) : EF_JPEG_E_CORRUPT;
      if (f.st != 0) SS[t].resize(f.seg_beg);
      f.seg_end = (int)SS[t].size();
    }
  };
  std::vector<int> t_beg(nt + 1);
  for (int t = 0; t <= nt; ++t) t_beg[t] = (int)((int64_t)count * t / nt);
  host_parallel(nt, [&](int t) { work(t, t_beg[t], t_beg[t + 1]); });
  // merge in file order: thread-local table indices -> batch tables, then the layout
  for (int t = 0; t < nt; ++t) {
    // tables enter the batch lazily, in the order the accepted files use them
    std::vector<int> hmap(TT[t].huff.size(), -1), qmap(TT[t].quant.size() / 64, -1);
    auto H = [&](int j) {
      if (hmap[j] < 0) hmap[j] = B.T.merge_huff(*TT[t].huff_key[j], TT[t].huff[j]);
      return hmap[j];
    };
    auto Q = [&](int j) {
      if (qmap[j] < 0) qmap[j] = B.T.quant_table(TT[t].quant.data() + 64 * j);
      return qmap[j];
    };
    for (int i = t_beg[t]; i < t_beg[t + 1]; ++i) {
      FileRes& f = R[i];
      JImage& im = f.im;
      int st = f.st;
      if (st == 0) {
        for (int k = 0; k < im.nc; ++k) {
          im.c[k].dc = H(im.c[k].dc);
          im.c[k].ac = H(im.c[k].ac);
        }
        for (int k = 0; k < im.nc; ++k) im.c[k].q = Q(im.c[k].q);
      }
      if (st == 0 && (int64_t)im.w * im.h > ((int64_t)1 << 31)) st = EF_JPEG_E_UNSUPPORTED;
      if (st == 0 && B.T.huff.size() >= (size_t)kMaxTables) st = EF_JPEG_E_UNSUPPORTED;  // int32 table offsets
      if (status) status[i] = st;
      if (st != 0) continue;
      for (int k = f.seg_beg; k < f.seg_end; ++k) {  // destuffed bytes never exceed the raw ones
        JSeg sg = SS[t][k];
        sg.img = (int)B.imgs.size();
        sg.word_off = B.words;
        B.words += (sg.end - sg.beg + 3) / 4 + 1;
        B.segs.push_back(sg);
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
      B.row_start.push_back(B.rows);
      B.rows += im.h;
      B.img_of.push_back(i);
      B.imgs.push_back(im);
    }
  }
}

// Copy segment sg's entropy bytes without the 0xFF00 stuffing into dst (zero-padded to a
// whole word); stops at the first marker, as jdhuff.c's fill_bit_buffer does.  Sets nbits.
void destuff(const uint8_t* src, int64_t n, JSeg& sg, uint8_t* dst) {
  int64_t q = 0, o = 0;
  while (q < n) {
    const void* f = std::memchr(src + q, 0xFF, (size_t)(n - q));
    const int64_t run = f ? static_cast<const uint8_t*>(f) - (src + q) : n - q;
    std::memcpy(dst + o, src + q, (size_t)run);
    o += run;
    q += run;
    if (!f) break;
    if (q + 1 < n && src[q + 1] == 0x00) {  // stuffed 0xFF
      dst[o++] = 0xFF;
      q += 2;
      continue;
    }
    break;  // a marker (or 0xFF fill before one, or a lone trailing 0xFF)
  }
  const int64_t padded = (o + 3) / 4 * 4 + 4;
  std::memset(dst + o, 0, (size_t)(padded - o));
  sg.nbits = (int)(o * 8);
}

// segments [s0, s1) of the batch (all of them: destuff_all)
void destuff_range(Batch& B, const uint8_t* data, const int64_t* offsets, uint8_t* words, size_t s0, size_t s1) {
  const size_t n = s1 - s0;
  auto work = [&](size_t a, size_t e) {
    for (size_t k = a; k < e; ++k) {
      JSeg& sg = B.segs[k];
      const uint8_t* file = data + offsets[B.img_of[sg.img]];
      destuff(file + sg.beg, sg.end - sg.beg, sg, words + sg.word_off * 4);
    }
  };
  const int64_t bytes = ((s1 < B.segs.size() ? B.segs[s1].word_off : B.words) - (n ? B.segs[s0].word_off : 0)) * 4;
  const size_t nt = bytes < ((int64_t)4 << 20) ? 1 : std::min<size_t>((size_t)host_threads(), n);
  host_parallel((int)nt, [&](int t) { work(s0 + n * t / nt, s0 + n * (t + 1) / nt); });
}
void destuff_all(Batch& B, const uint8_t* data, const int64_t* offsets, uint8_t* words) {
  destuff_range(B, data, offsets, words, 0, B.segs.size());
}

// Chunk size: about 128k chunks for the batch (4 per SIMD lane group of the chip), kept in
// [2048, 16384] bits so self-synchronisation stays a small fraction of each chunk.
void make_chunks(Batch& B, int64_t opt_bits) {
  int64_t total = 0;
  for (const JSeg& sg : B.segs) total += sg.nbits;
  int64_t cb = opt_bits > 0 ? opt_bits : (total / 131072 + 255) / 256 * 256;
  cb = std::max<int64_t>(opt_bits > 0 ? 64 : 2048, std::min<int64_t>(cb, 16384));
  B.chunk_bits = (int)cb;
  B.warm_bits = (int)std::min<int64_t>(cb, 1024);
  B.chunk_seg.clear();
  for (size_t k = 0; k < B.segs.size(); ++k) {
    JSeg& sg = B.segs[k];
    sg.chunk0 = (int)B.chunk_seg.size();
    sg.nchunk = (int)std::max<int64_t>(1, (sg.nbits + cb - 1) / cb);
    B.chunk_seg.insert(B.chunk_seg.end(), sg.nchunk, (int)k);
  }
}

// A built batch staged for upload: one pinned slot holds [destuffed words | images |
// Huffman tables | quant tables | segments | IDCT runs | pixel starts | file -> image map |
// chunk table]; the chunk table is cut after destuffing, into room reserved for its bound.
// The slot uploads as one copy of up_bytes into the device slot of the same index.
struct Staged {
  int slot = 0;
  char* h = nullptr;
  size_t o_words = 0, o_imgs = 0, o_pool = 0, o_q = 0, o_seg = 0, o_bs = 0, o_ic = 0, o_ps = 0, o_desc = 0, o_cseg = 0;
  size_t pin_need = 0, up_bytes = 0;
  size_t words_up = 0;  // leading bytes already uploaded into the device slot (early upload)
};

// Host half of a decode: size / allocate pinned slot `slot` (waiting for the upload that last
// read it), destuff the entropy segments into it, copy the tables, cut the chunks.  Touches
// only this slot and B, so it may run on a host thread while another slot's batch decodes.
// Returns EF_OK, or an error code with the message in *err (the caller records it).
int jpeg_ensure(ef_ctx* c, DevBuf& b, size_t bytes);
hipError_t jpeg_event(hipEvent_t* ev, hipStream_t record_on);
constexpr int kUploadPhases = 4;  // early upload: destuff + upload pieces per batch
bool jpeg_early_upload() {
#ifdef EF_DIAGNOSTICS  // EF_JPEG_EARLY_UP=0: the whole upload after staging, round 5's order (A/B)
  if (const char* e = getenv("EF_JPEG_EARLY_UP")) return atoi(e) != 0;
#endif
  return true;
}
int stage_batch(ef_ctx* c, int slot, Batch& B, const uint8_t* data, const int64_t* offsets, Staged& S,
                std::string* err, int64_t chunk_bits = 0, bool early_upload = false) {
  StageTimer tm;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  size_t off = 0;
  S.slot = slot;
  S.o_words = off; off += al((size_t)B.words * 4 + 32);  // BitStream reads up to 8 words past a segment
  S.o_imgs = off; off += al(B.imgs.size() * sizeof(JImage));
  S.o_pool = off; off += al(std::max<size_t>(B.T.huff.size(), 1) * sizeof(HuffTab));
  S.o_q = off; off += al(std::max<size_t>(B.T.quant.size(), 1) * 2);
  S.o_seg = off; off += al(B.segs.size() * sizeof(JSeg));
  S.o_bs = off; off += al(B.block_start.size() * 8);
  S.o_ic = off; off += al(B.ic.size() * 4);
  S.o_ps = off; off += al(B.row_start.size() * 8);
  S.o_desc = off; off += al(B.file_img.size() * 4);
  S.o_cseg = off;  // chunk table last: its size is known only after destuffing
  {  // make_chunks' bound: every segment has <= nbits / chunk_bits + 1 chunks
    const int64_t cb_min = (c->opt_jpeg_chunk_bits > 0 || chunk_bits > 0) ? 64 : 2048;
    off += al(((size_t)(B.words * 32 / cb_min) + B.segs.size() + 1) * 4);
  }
  S.pin_need = off;
  if (c->jpeg_up_done[slot]) {  // the upload that last read this slot
    const hipError_t e = hipEventSynchronize(c->jpeg_up_done[slot]);
    if (e != hipSuccess) { *err = hipGetErrorString(e); return EF_E_HIP; }
  }
  if (c->jpeg_pinned_bytes[slot] < S.pin_need) {
    if (c->jpeg_pinned[slot]) (void)hipHostFree(c->jpeg_pinned[slot]);
    c->jpeg_pinned[slot] = nullptr;
    c->jpeg_pinned_bytes[slot] = 0;
    const size_t want = S.pin_need + S.pin_need / 4 + 4096;
    const hipError_t e = hipHostMalloc(&c->jpeg_pinned[slot], want, hipHostMallocDefault);
    if (e != hipSuccess) {
      c->jpeg_pinned[slot] = nullptr;
      *err = std::string("hipHostMalloc (jpeg staging): ") + hipGetErrorString(e);
      return EF_E_HIP;
    }
    c->jpeg_pinned_bytes[slot] = want;
  }
  char* h = static_cast<char*>(c->jpeg_pinned[slot]);
  S.h = h;
  tm.mark("pinned");
  S.words_up = 0;
  // The destuffed words go up in kUploadPhases pieces as they are produced (copy stream,
  // behind the kernels that last read this device slot), so a batch's upload overlaps its
  // own destuffing instead of following the whole host staging; launch_batch uploads the
  // rest (padding, tables, chunk table).  Only into a device slot already large enough
  // (launch_batch sizes slots by pin_need; this may run on a staging thread, which must
  // not reallocate): the first call at a new size uploads whole, as without early upload.
  if (early_upload && c->jpeg_copy && !B.segs.empty() && c->jpeg_up[slot].p &&
      c->jpeg_up[slot].bytes >= S.pin_need + 16) {
    hipError_t e = jpeg_event(&c->jpeg_ws_free[slot], c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->jpeg_copy, c->jpeg_ws_free[slot], 0);
    char* up = static_cast<char*>(c->jpeg_up[slot].p);
    const size_t nseg = B.segs.size();
    for (int ph = 0; ph < kUploadPhases && e == hipSuccess; ++ph) {
      const size_t a = nseg * ph / kUploadPhases, b = nseg * (ph + 1) / kUploadPhases;
      if (a == b) continue;
      destuff_range(B, data, offsets, reinterpret_cast<uint8_t*>(h + S.o_words), a, b);
      const size_t w0 = (size_t)B.segs[a].word_off * 4, w1 = (size_t)(b < nseg ? B.segs[b].word_off : B.words) * 4;
      e = hipMemcpyAsync(up + S.o_words + w0, h + S.o_words + w0, w1 - w0, hipMemcpyHostToDevice, c->jpeg_copy);
    }
    if (e != hipSuccess) {  // (pieces already queued must not outlive the pinned slot's next use)
      *err = hipGetErrorString(e);
      (void)hipStreamSynchronize(c->jpeg_copy);
      return EF_E_HIP;
    }
    S.words_up = S.o_words + (size_t)B.words * 4;
  } else {
    destuff_all(B, data, offsets, reinterpret_cast<uint8_t*>(h + S.o_words));
  }
  tm.mark("destuff");
  make_chunks(B, c->opt_jpeg_chunk_bits > 0 ? c->opt_jpeg_chunk_bits : chunk_bits);
  std::memcpy(h + S.o_imgs, B.imgs.data(), B.imgs.size() * sizeof(JImage));
  if (!B.T.huff.empty()) std::memcpy(h + S.o_pool, B.T.huff.data(), B.T.huff.size() * sizeof(HuffTab));
  if (!B.T.quant.empty()) std::memcpy(h + S.o_q, B.T.quant.data(), B.T.quant.size() * 2);
  std::memcpy(h + S.o_seg, B.segs.data(), B.segs.size() * sizeof(JSeg));
  std::memcpy(h + S.o_bs, B.block_start.data(), B.block_start.size() * 8);
  std::memcpy(h + S.o_ic, B.ic.data(), B.ic.size() * 4);
  std::memcpy(h + S.o_ps, B.row_start.data(), B.row_start.size() * 8);
  if (!B.file_img.empty()) std::memcpy(h + S.o_desc, B.file_img.data(), B.file_img.size() * 4);
  std::memcpy(h + S.o_cseg, B.chunk_seg.data(), B.chunk_seg.size() * 4);
  S.up_bytes = S.o_cseg + B.chunk_seg.size() * 4;
  tm.mark("tables");
  return EF_OK;
}

// ensure() for the buffers a queued decode may still use: a reallocation first waits for
// the context's queued uploads and decodes (growth only; steady-state calls never wait).
int jpeg_ensure(ef_ctx* c, DevBuf& b, size_t bytes) {
  if (b.p && b.bytes >= bytes) return EF_OK;
  const hipError_t e = jpeg_quiesce(c);
  if (e != hipSuccess) return hip_err(c, e, "jpeg decode");
  return ensure(c, b, bytes);
}

hipError_t jpeg_event(hipEvent_t* ev, hipStream_t record_on) {
  if (*ev) return hipSuccess;
  hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (e == hipSuccess && record_on) e = hipEventRecord(*ev, record_on);  // waits on it pass until re-recorded
  return e;
}

// Device half: upload a staged batch (copy stream), entropy-decode and IDCT it, then either
// colour-convert it into dout (device), each image at its out_off, or — for the ingest
// (rz_dst) — resize every file of the batch to an (oh x ow) grey row of rz_dst straight from
// the planes (jpeg_resize_kernel, file -> image map staged with the batch).
// Stream-ordered on ctx's stream and never waits on the host: the synchronisation rounds
// are queued back to back (a round after the fixed point exits at once) and a batch that
// has not converged after them is completed on the device (jpeg_finish_kernel).
int launch_batch(ef_ctx* c, Batch& B, const Staged& S, uint8_t* dout, uint8_t* rz_dst = nullptr, int oh = 0,
                 int ow = 0) {
  hipStream_t s = c->stream;
  StageTimer tm;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const int slot = S.slot;
  const int nchunks = (int)B.chunk_seg.size();
  size_t off = 0;
  const size_t o_S = off; off += al((size_t)nchunks * 8);
  const size_t o_E0 = off; off += al((size_t)nchunks * 8);
  const size_t o_E1 = off; off += al((size_t)nchunks * 8);
  const size_t o_cnt = off; off += al((size_t)nchunks * 16);
  const size_t o_G = off; off += al((size_t)nchunks * 4);
  const size_t o_P = off; off += al((size_t)nchunks * 12);
  const size_t o_flag = off; off += al(4 * (kDeviceRounds + 2));
  const size_t o_cps = off; off += al((size_t)nchunks * kCheckpoints * sizeof(Checkpoint));
  const size_t o_coef = off; off += al((size_t)B.coef_blocks * 64 * 2);
  const size_t o_planes = off; off += al((size_t)B.plane_bytes + 16);
  hipError_t e = hipSuccess;
  if (!c->jpeg_copy) e = hipStreamCreateWithFlags(&c->jpeg_copy, hipStreamNonBlocking);
  if (e == hipSuccess) e = jpeg_event(&c->jpeg_up_done[slot], nullptr);
  if (e == hipSuccess) e = jpeg_event(&c->jpeg_ws_free[slot], s);
  if (e == hipSuccess) e = jpeg_event(&c->jpeg_done, s);
  if (e != hipSuccess) return hip_err(c, e, "jpeg decode");
  {
    int rc = jpeg_ensure(c, c->jpeg_ws, off);
    if (rc == EF_OK) rc = jpeg_ensure(c, c->jpeg_up[slot], std::max(S.pin_need, S.up_bytes) + 16);
    if (rc != EF_OK) return rc;
  }
  char* up = static_cast<char*>(c->jpeg_up[slot].p);
  char* base = static_cast<char*>(c->jpeg_ws.p);
  // upload on the copy stream once the kernels that last read this device slot are done;
  // the compute stream waits for it and for the previous decode (shared workspace)
  hipStream_t cs = c->jpeg_copy;
  e = hipStreamWaitEvent(cs, c->jpeg_ws_free[slot], 0);
  if (e == hipSuccess)  // (the words went up already with an early upload: the rest)
    e = hipMemcpyAsync(up + S.words_up, S.h + S.words_up, S.up_bytes - S.words_up, hipMemcpyHostToDevice, cs);
  if (e == hipSuccess) e = hipEventRecord(c->jpeg_up_done[slot], cs);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, c->jpeg_up_done[slot], 0);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, c->jpeg_done, 0);
  tm.mark("upload", cs, true);
  TimerEvt tev;
  timer_begin(c, EF_KERNEL_JPEG, &tev);
  if (e == hipSuccess) e = hipMemsetAsync(base + o_coef, 0, (size_t)B.coef_blocks * 64 * 2, s);
  ChunkCtx X;
  X.chunk_seg = reinterpret_cast<const int*>(up + S.o_cseg);
  X.segs = reinterpret_cast<const JSeg*>(up + S.o_seg);
  X.imgs = reinterpret_cast<const JImage*>(up + S.o_imgs);
  X.pool = reinterpret_cast<const HuffTab*>(up + S.o_pool);
  X.words = reinterpret_cast<const unsigned*>(up + S.o_words);
  X.nchunks = nchunks;
  X.chunk_bits = B.chunk_bits;
  X.warm_bits = B.warm_bits;
  X.cps = reinterpret_cast<Checkpoint*>(base + o_cps);
  long long* S_ = reinterpret_cast<long long*>(base + o_S);
  long long* E[2] = {reinterpret_cast<long long*>(base + o_E0), reinterpret_cast<long long*>(base + o_E1)};
  int* cnt = reinterpret_cast<int*>(base + o_cnt);
  int* G = reinterpret_cast<int*>(base + o_G);
  int* P = reinterpret_cast<int*>(base + o_P);
  int* flag = reinterpret_cast<int*>(base + o_flag);
  int max_chunks = 1;
  for (const JSeg& sg : B.segs) max_chunks = std::max(max_chunks, sg.nchunk);
  const unsigned cgrid = (unsigned)((nchunks + kChunkThreads - 1) / kChunkThreads);
  const int lds_tables = B.T.huff.size() <= (size_t)kLdsTables ? (int)B.T.huff.size() : 0;
  const size_t lds_bytes = (size_t)lds_tables * kTabBytes;
  if (e == hipSuccess) {  // up to kLdsTables whole tables: > 64 KiB of dynamic LDS
    const int most = kLdsTables * kTabBytes + 128;
    e = allow_dynamic_lds(reinterpret_cast<const void*>(jpeg_sync_kernel), most);
    if (e == hipSuccess) e = allow_dynamic_lds(reinterpret_cast<const void*>(jpeg_write_kernel), most);
  }
  const int nseg = (int)B.segs.size();
  // flag[r]: round r changed an exit state (r = 1 .. kDeviceRounds)
  if (e == hipSuccess) e = hipMemsetAsync(flag, 0, 4 * (kDeviceRounds + 2), s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(jpeg_sync_kernel, dim3(cgrid), dim3(kChunkThreads), lds_bytes, s, X, lds_tables, 0, S_, E[1],
                       E[0], cnt, flag, nullptr);
    e = hipGetLastError();
  }
  // Synchronisation rounds until no start state changes.  Round r makes chunk r of every
  // segment exact, so a segment of m chunks needs at most m - 1; the first kDeviceRounds
  // are queued back to back, and jpeg_finish_kernel completes whatever has not converged
  // after them (nothing, in the test corpora and the bench set: 3-4 rounds).
  int cur = 0;
  const int qrounds = std::min(max_chunks, kDeviceRounds);
  for (int r = 1; e == hipSuccess && r <= qrounds; ++r) {
    hipLaunchKernelGGL(jpeg_sync_kernel, dim3(cgrid), dim3(kChunkThreads), lds_bytes, s, X, lds_tables, r, S_, E[cur],
                       E[cur ^ 1], cnt, flag + r, r >= 2 ? flag + r - 1 : nullptr);
    e = hipGetLastError();
    cur ^= 1;
  }
  if (e == hipSuccess && max_chunks > qrounds) {
    hipLaunchKernelGGL(jpeg_finish_kernel, dim3((unsigned)((nseg + 63) / 64)), dim3(64), 0, s, X, nseg, qrounds, S_,
                       E[cur], cnt, flag + qrounds);
    e = hipGetLastError();
  }
  tm.mark("sync-rounds", s, true);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(jpeg_scan_kernel, dim3((unsigned)((nseg + 63) / 64)), dim3(64), 0, s, X, nseg, cnt, G, P);
    hipLaunchKernelGGL(jpeg_write_kernel, dim3(cgrid), dim3(kChunkThreads), lds_bytes + 128, s, X, lds_tables, S_, G,
                       P, reinterpret_cast<short*>(base + o_coef));
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    const JImage* d_imgs = X.imgs;
    short* d_coef = reinterpret_cast<short*>(base + o_coef);
    uint8_t* d_planes = reinterpret_cast<uint8_t*>(base + o_planes);
    if (B.blocks > 0)
      hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((B.blocks + kIdctBlocks - 1) / kIdctBlocks)), dim3(256), 0,
                         s, d_coef, d_imgs, reinterpret_cast<const int64_t*>(up + S.o_bs), (int)B.block_start.size(),
                         reinterpret_cast<const int*>(up + S.o_ic), reinterpret_cast<const unsigned short*>(up + S.o_q),
                         B.blocks, d_planes);
    if (B.rows > 0 && !rz_dst)
      hipLaunchKernelGGL(jpeg_out_kernel, dim3((unsigned)((B.rows + 3) / 4)), dim3(256), 0, s, d_imgs,
                         reinterpret_cast<const int64_t*>(up + S.o_ps), (int)B.imgs.size(), B.rows, d_planes, dout);
    e = hipGetLastError();
  }
  timer_end(c, &tev);
  if (e == hipSuccess && rz_dst && !B.file_img.empty()) {
    TimerEvt tr;
    timer_begin(c, EF_KERNEL_INGEST, &tr);
    hipLaunchKernelGGL(jpeg_resize_kernel, dim3((unsigned)((oh + kResizeBand - 1) / kResizeBand), (unsigned)B.file_img.size()),
                       dim3(256), 0, s, X.imgs, reinterpret_cast<const int*>(up + S.o_desc),
                       reinterpret_cast<const uint8_t*>(base + o_planes), oh, ow, rz_dst);
    e = hipGetLastError();
    timer_end(c, &tr);
  }
  if (e == hipSuccess) e = hipEventRecord(c->jpeg_ws_free[slot], s);
  if (e == hipSuccess) e = hipEventRecord(c->jpeg_done, s);
  tm.mark("kernels", s, true);
  if (e != hipSuccess) return hip_err(c, e, "jpeg decode");
  return EF_OK;
}


// Host and device halves in sequence (the context's next slot).
int decode_batch(ef_ctx* c, Batch& B, const uint8_t* data, const int64_t* offsets, uint8_t* dout) {
  Staged S;
  std::string err;
  const int slot = c->jpeg_slot;
  c->jpeg_slot ^= 1;
  const int rc = stage_batch(c, slot, B, data, offsets, S, &err);
  if (rc != EF_OK) return set_err(c, rc, "jpeg decode: " + err);
  return launch_batch(c, B, S, dout);
}

}  // namespace

hipError_t jpeg_quiesce(ef_ctx* c) {
  hipError_t e = hipSuccess;
  if (c->jpeg_done) e = hipEventSynchronize(c->jpeg_done);
  if (e == hipSuccess && c->jpeg_copy) e = hipStreamSynchronize(c->jpeg_copy);
  return e;
}

}  // namespace ef

using namespace ef;

extern "C" {

int ef_jpeg_info(const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count, int32_t* heights,
                 int32_t* widths, int32_t* components, int32_t* status) {
  if (count < 0 || (count > 0 && (!data || !offsets || !sizes))) return EF_E_INVALID;
  Tables T;
  std::vector<JSeg> segs;
  for (int i = 0; i < count; ++i) {
    JImage im{};
    int st = sizes[i] > 0 ? parse(data + offsets[i], sizes[i], i, im, T, segs, false) : EF_JPEG_E_CORRUPT;
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
  const bool dev_out = (flags & EF_MEM_DEVICE) != 0;
  const int ch = mode == EF_JPEG_GRAY ? 1 : 3;
  Batch B;
  build_batch(data, offsets, sizes, count, mode, dev_out ? out_offsets : nullptr, status, B);
  if (B.imgs.empty()) return EF_OK;
  uint8_t* dout = out;
  if (!dev_out) {
    const int rc = ensure(c, c->jpeg_out, (size_t)B.dense_out + 16);
    if (rc != EF_OK) return rc;
    dout = static_cast<uint8_t*>(c->jpeg_out.p);
  }
  const int rc = decode_batch(c, B, data, offsets, dout);
  if (rc != EF_OK || dev_out) return rc;  // device output: stream-ordered like other EF_MEM_DEVICE calls
  std::vector<uint8_t> dense((size_t)B.dense_out);
  hipError_t e = hipMemcpyAsync(dense.data(), dout, (size_t)B.dense_out, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
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
#ifdef EF_DIAGNOSTICS  // EF_JPEG_CALLTIMES: per call, host ms of the staging and of the whole call (no syncs)
  struct CallClock {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    bool on = std::getenv("EF_JPEG_CALLTIMES") != nullptr;
    double prep = 0.0;
    ~CallClock() {
      if (on)
        std::fprintf(stderr, "[ingest] prepare %.3f ms, call %.3f ms\n", prep,
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
  } call_clock;
#endif
  (void)hipSetDevice(c->device);
  if (!c->jpeg_copy) {  // (created here, before any staging thread can use it)
    const hipError_t e = hipStreamCreateWithFlags(&c->jpeg_copy, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_err(c, e, "jpeg ingest");
  }
  const int64_t row = (int64_t)out_h * out_w;
  // Parts of ~kIngestPart files, each staged (parse, destuff, tables, chunks, file -> image
  // map) into one of the context's two upload slots, the next part on a host thread
  // while this one is queued.  Nothing in a part's device work waits on the host (see
  // launch_batch), so with device output the call returns once every part is queued, and
  // the next call's host staging overlaps this call's decode.
  // Parts keep the whole call's entropy-chunk size (a part sized on its own would cut
  // twice as many, shorter chunks, whose warm-up and synchronisation cost more than the
  // overlap wins).  Calls up to EF_OPT_JPEG_PART_FILES (8192) files run as one part.
  const int32_t kIngestPart = (int32_t)std::max<int64_t>(1, c->opt_jpeg_part_files);
  struct Part {
    int32_t a = 0, m = 0;
    int slot = 0;
    Batch B;
    Staged S;
    std::vector<int32_t> st;
    int rc = EF_OK;
    std::string err;
    double host_ms = 0.0;  // wall time of prepare() (EF_KERNEL_JPEG_HOST)
  };
  int64_t call_chunk_bits = 0;
  auto prepare = [&](Part& P) {
    (void)hipSetDevice(c->device);  // a fresh host thread starts on device 0
    struct Stamp {  // every return path records the part's host time
      Part& P;
      std::chrono::steady_clock::time_point t0;
      ~Stamp() { P.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } stamp{P, std::chrono::steady_clock::now()};
    StageTimer tm;
    P.st.assign(P.m, 0);
    build_batch(data, offsets + P.a, sizes + P.a, P.m, mode, nullptr, P.st.data(), P.B);
    tm.mark("parse");
    if (P.B.imgs.empty()) return;
    Batch& B = P.B;
    B.file_img.assign((size_t)P.m, -1);  // file j of the part -> row j
    for (size_t q = 0; q < B.imgs.size(); ++q) B.file_img[(size_t)B.img_of[q]] = (int)q;
    P.rc = stage_batch(c, P.slot, B, data, offsets + P.a, P.S, &P.err, call_chunk_bits, jpeg_early_upload());
  };
  for (int32_t a0 = 0; a0 < count; a0 += 65535) {  // the resize launch's per-launch image limit
    const int32_t m0 = std::min<int32_t>(65535, count - a0);
    uint8_t* rows_all = out + (int64_t)a0 * row;
    if (!(flags & EF_MEM_DEVICE)) {  // host rows: resize into device staging, then copy out
      const int rc = jpeg_ensure(c, c->jpeg_rows, (size_t)m0 * row);
      if (rc != EF_OK) return rc;
      rows_all = static_cast<uint8_t*>(c->jpeg_rows.p);
    }
    const int32_t nparts = (m0 + kIngestPart - 1) / kIngestPart;
    // make_chunks' rule on the call's file bytes (entropy bits ~ file bytes x 8)
    int64_t bytes = 0;
    for (int32_t i = 0; i < m0; ++i) bytes += std::max<int64_t>(sizes[a0 + i], 0);
    call_chunk_bits = nparts > 1 ? std::max<int64_t>(2048, std::min<int64_t>((bytes * 8 / 131072 + 255) / 256 * 256, 16384)) : 0;
    std::vector<Part> parts(nparts);
    for (int32_t i = 0; i < nparts; ++i) {
      parts[i].a = a0 + (int32_t)((int64_t)m0 * i / nparts);
      parts[i].m = a0 + (int32_t)((int64_t)m0 * (i + 1) / nparts) - parts[i].a;
      parts[i].slot = c->jpeg_slot;
      c->jpeg_slot ^= 1;
    }
    prepare(parts[0]);
    for (int32_t i = 0; i < nparts; ++i) {
      Part& P = parts[i];
      std::thread next;
      if (i + 1 < nparts) next = std::thread(prepare, std::ref(parts[i + 1]));
      int rc = P.rc != EF_OK ? set_err(c, P.rc, "ef_jpeg_ingest: " + P.err) : EF_OK;
      uint8_t* dst = rows_all + (int64_t)(P.a - a0) * row;
      if (rc == EF_OK && P.B.imgs.empty()) {  // no file of the part decodes here: zero rows
        const hipError_t e = hipMemsetAsync(dst, 0, (size_t)P.m * row, c->stream);
        if (e != hipSuccess) rc = hip_err(c, e, "jpeg ingest");
      } else if (rc == EF_OK) {
        rc = launch_batch(c, P.B, P.S, nullptr, dst, out_h, out_w);
      }
      if (next.joinable()) next.join();  // before any return: the thread uses parts[i + 1]
      if (rc != EF_OK) return rc;
      if (status) std::memcpy(status + P.a, P.st.data(), (size_t)P.m * 4);
#ifdef EF_DIAGNOSTICS
      call_clock.prep += P.host_ms;
#endif
      if (c->timing) {  // host staging time of this part (recorded on the calling thread)
        c->t_ms[EF_KERNEL_JPEG_HOST] += P.host_ms;
        c->t_n[EF_KERNEL_JPEG_HOST] += 1;
      }
      P.B = Batch();  // release the part's host tables
    }
    if (!(flags & EF_MEM_DEVICE)) {
      hipError_t e = hipMemcpyAsync(out + (int64_t)a0 * row, rows_all, (size_t)m0 * row, hipMemcpyDeviceToHost,
                                    c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) return hip_err(c, e, "jpeg ingest");
    }
  }
  return EF_OK;
}

}  // extern "C"


#ifdef EF_DIAGNOSTICS
// Diagnostic build only (never loaded by the package): the same per-thread device
// functions run in host loops, so decoder changes can be checked on a machine without
// a GPU (tools/micro/jpeg_host_check.py).  Output layout as ef_jpeg_decode's host form;
// *rounds_out receives the number of synchronisation rounds.
extern "C" int ef_diag_jpeg_decode_host(const uint8_t* data, const int64_t* offsets, const int64_t* sizes,
                                        int32_t count, int32_t mode, uint8_t* out, const int64_t* out_offsets,
                                        int32_t* status, int32_t chunk_bits, int32_t* rounds_out) {
  Batch B;
  build_batch(data, offsets, sizes, count, mode, out_offsets, status, B);
  std::vector<unsigned> words((size_t)B.words + 16, 0);  // BitStream's block reads run ahead
  destuff_all(B, data, offsets, reinterpret_cast<uint8_t*>(words.data()));
  make_chunks(B, chunk_bits);
  const int nch = (int)B.chunk_seg.size();
  std::vector<Checkpoint> cps((size_t)nch * kCheckpoints);
  ChunkCtx X{B.chunk_seg.data(), B.segs.data(), B.imgs.data(), B.T.huff.data(), words.data(), nch, B.chunk_bits,
             B.warm_bits, cps.data()};
  std::vector<long long> S(nch), E0(nch), E1(nch);
  std::vector<int> cnt((size_t)nch * 4), G(nch), P((size_t)nch * 3);
  int changed = 0;
  const unsigned short* luts = B.T.huff.empty() ? nullptr : B.T.huff[0].look;
  const int ls = kGlobalLutStride;
  for (int i = 0; i < nch; ++i)
    sync_chunk(X, X.pool, luts, ls, i, 0, S.data(), E1.data(), E0.data(), cnt.data(), &changed);
  long long* Ein = E0.data();
  long long* Eout = E1.data();
  int rounds = 0;
  // EF_JPEG_QROUNDS=q: stop after q rounds and complete with finish_segment, as the device
  // does after its queued rounds
  const char* qenv = std::getenv("EF_JPEG_QROUNDS");
  const int qmax = qenv ? std::max(1, std::atoi(qenv)) : nch + 1;
  for (int r = 1; r <= std::min(qmax, nch + 1); ++r) {
    changed = 0;
    const std::vector<long long> S0 = S;
    for (int i = 0; i < nch; ++i) sync_chunk(X, X.pool, luts, ls, i, r, S.data(), Ein, Eout, cnt.data(), &changed);
    int nchg = 0;
    for (int i = 0; i < nch; ++i) nchg += S[i] != S0[i];
    std::fprintf(stderr, "round %d: %d of %d chunk starts changed\n", r, nchg, nch);
    std::swap(Ein, Eout);
    rounds = r;
    if (!changed) break;
  }
  if (changed) {
    for (const JSeg& sg : B.segs) finish_segment(X, luts, ls, sg, rounds, S.data(), Ein, cnt.data());
    std::fprintf(stderr, "finished after %d rounds\n", rounds);
  }
  if (rounds_out) *rounds_out = rounds;
  if (std::getenv("EF_JPEG_CHECK")) {  // recompute every non-last chunk's counts and exit from its start
    int bad = 0;
    for (int i = 0; i < nch; ++i) {
      const JSeg& sg = B.segs[B.chunk_seg[i]];
      const int j = i - sg.chunk0;
      if (j == sg.nchunk - 1) continue;
      McuInfo M;
      M.load(B.imgs[sg.img]);
      BitStream bs;
      chunk_stream(X, sg, st_pos(S[i]), bs);
      int c4[4];
      const long long e = chunk_sync(M, X.pool, luts, ls, bs, st_b(S[i]), st_k(S[i]), (j + 1) * X.chunk_bits, c4);
      if (e != Ein[i] || c4[0] != cnt[4 * i] || c4[1] != cnt[4 * i + 1] || c4[2] != cnt[4 * i + 2] ||
          c4[3] != cnt[4 * i + 3] || (j + 1 < sg.nchunk && S[i + 1] != e)) {
        if (bad++ < 5)
          std::fprintf(stderr, "chunk %d (seg %d j %d): exit %lld vs %lld, n %d vs %d, next S %lld\n", i,
                       B.chunk_seg[i], j, e, Ein[i], c4[0], cnt[4 * i], S[i + 1]);
      }
    }
    std::fprintf(stderr, "check: %d bad chunks\n", bad);
  }
  for (const JSeg& sg : B.segs) scan_segment(X, sg, cnt.data(), G.data(), P.data());
  std::vector<short> coef((size_t)B.coef_blocks * 64 + 64, 0);
  for (int i = 0; i < nch; ++i)
    write_chunk(X, X.pool, luts, ls, i, S.data(), G.data(), P.data(), coef.data(), kNaturalHost);
  std::vector<uint8_t> planes((size_t)B.plane_bytes + 16);
  for (size_t r = 0; r < B.block_start.size(); ++r) {
    const JImage& im = B.imgs[B.ic[r] >> 2];
    const JComp& cp = im.c[B.ic[r] & 3];
    const unsigned short* q = B.T.quant.data() + (int64_t)(im.qt_base + cp.q) * 64;
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
    for (int y = 0; y < im.h; ++y)
      for (int x0 = 0; x0 < im.w; x0 += 4) out_quad(im, y, x0, planes.data(), out);
  return EF_OK;
}
// host preparation only (parse, destuff, chunking): wall time of each stage in ms
extern "C" int ef_diag_jpeg_prep_host(const uint8_t* data, const int64_t* offsets, const int64_t* sizes,
                                      int32_t count, int32_t mode, double* ms3) {
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const auto t0 = now();
  Batch B;
  build_batch(data, offsets, sizes, count, mode, nullptr, nullptr, B);
  std::vector<unsigned> words((size_t)B.words + 4, 0);
  const auto t1 = now();
  destuff_all(B, data, offsets, reinterpret_cast<uint8_t*>(words.data()));
  const auto t2 = now();
  make_chunks(B, 0);
  const auto t3 = now();
  ms3[0] = ms(t0, t1);
  ms3[1] = ms(t1, t2);
  ms3[2] = ms(t2, t3);
  return (int)B.T.huff.size();
}
#endif
