// mcpt_image.cpp — host half of the output step and the Transfo helpers
// of the C ABI.
//
//  * mcpt_average: the display pass fs_frag, accum / nb (MontecarloGPU/montecarlo.cpp:59-70,
//    470-476), one binary32 division per channel.
//  * mcpt_write_pfm: the averaged RGB32F image as a little-endian PFM (row 0 = bottom, which
//    is both GL's and PFM's row order).
//  * mcpt_write_png: what the default framebuffer shows: each channel clamped to [0,1] and
//    converted to 8-bit unorm by round(255·c) (GL float→unorm rule, no gamma), written as an
//    8-bit RGB PNG (top row first) with stored (uncompressed) deflate blocks.
//  * mcpt_checkpoint_write / _read: a progressive render's accumulator, pass count and next
//    first pass in one file, so the pass loop (montecarlo.cpp:454-466) can stop and resume;
//    mcpt_checkpoint_save / _load (mcpt_capi.hip) add the target's identity (H, row-list hash).
//  * mcpt_transfo_*, mcpt_mat4_mul: easycppogl Transfo (gl_eigen.cpp:29-105, degrees) and
//    Eigen's float product, evaluated with the same arithmetic as the scene producer, so a
//    C++ caller composing transforms gets the reference's matrices bit for bit.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "../../include/mcpt.h"

// mcpt_capi.hip: an error return without a detail (drops the thread's unread detail)
int mcpt_err_bare(int status);

namespace mcpt {
namespace host {
void transfo_translate(float x, float y, float z, float* out);
void transfo_scale(float x, float y, float z, float* out);
void transfo_rotate(int axis, float deg, float* out);
void mat4_mul(const float* a, const float* b, float* out);
}  // namespace host
}  // namespace mcpt

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

uint32_t crc32(const unsigned char* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  if (!crc_ready) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t v = i;
      for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
      crc_table[i] = v;
    }
    crc_ready = true;
  }
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}

void be32(std::vector<unsigned char>& o, uint32_t v) {
  o.push_back((unsigned char)(v >> 24)); o.push_back((unsigned char)(v >> 16));
  o.push_back((unsigned char)(v >> 8)); o.push_back((unsigned char)v);
}

void chunk(std::vector<unsigned char>& out, const char* type, const std::vector<unsigned char>& data) {
  be32(out, (uint32_t)data.size());
  std::vector<unsigned char> td(type, type + 4);
  td.insert(td.end(), data.begin(), data.end());
  out.insert(out.end(), td.begin(), td.end());
  be32(out, crc32(td.data(), td.size()) ^ 0xFFFFFFFFu);
}

unsigned char unorm8(float c) {
  if (!(c > 0.0f)) return 0;            // also NaN -> 0
  if (c >= 1.0f) return 255;
  return (unsigned char)std::lround((double)c * 255.0);
}

}  // namespace

extern "C" {

int mcpt_average(const float* accum, long long n_values, int pass_count, float* out) {
  if (!accum || !out || n_values < 0 || pass_count <= 0) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  const float nb = (float)pass_count;
  for (long long i = 0; i < n_values; ++i) out[i] = accum[i] / nb;
  return MCPT_OK;
}

int mcpt_write_pfm(const char* path, const float* rgb, int W, int H) {
  if (!path || !rgb || W <= 0 || H <= 0) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  FILE* f = std::fopen(path, "wb");
  if (!f) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  std::fprintf(f, "PF\n%d %d\n-1.0\n", W, H);   // negative scale = little endian
  const size_t n = (size_t)W * H * 3;
  const bool ok = std::fwrite(rgb, sizeof(float), n, f) == n;
  return (std::fclose(f) == 0 && ok) ? MCPT_OK : MCPT_ERR_INVALID_ARG;
}

int mcpt_write_png(const char* path, const float* rgb, int W, int H) {
  if (!path || !rgb || W <= 0 || H <= 0 || W > (1 << 24) || H > (1 << 24)) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  // raw scanlines, filter 0, top row first (the accumulator's row 0 is the bottom)
  const size_t row = (size_t)W * 3 + 1;
  std::vector<unsigned char> raw(row * H);
  for (int y = 0; y < H; ++y) {
    unsigned char* r = &raw[(size_t)y * row];
    r[0] = 0;
    const float* src = rgb + (size_t)(H - 1 - y) * W * 3;
    for (int i = 0; i < W * 3; ++i) r[1 + i] = unorm8(src[i]);
  }
  // zlib stream of stored blocks (≤ 65535 bytes each) + adler32
  std::vector<unsigned char> z = {0x78, 0x01};
  size_t pos = 0;
  do {
    const size_t len = std::min<size_t>(65535, raw.size() - pos);
    const bool last = pos + len == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((unsigned char)(len & 0xFF)); z.push_back((unsigned char)(len >> 8));
    z.push_back((unsigned char)(~len & 0xFF)); z.push_back((unsigned char)((~len >> 8) & 0xFF));
    z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + len);
    pos += len;
  } while (pos < raw.size());
  uint32_t a = 1, b = 0;
  for (unsigned char c : raw) { a = (a + c) % 65521; b = (b + a) % 65521; }
  be32(z, (b << 16) | a);

  std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<unsigned char> ihdr;
  be32(ihdr, (uint32_t)W); be32(ihdr, (uint32_t)H);
  ihdr.push_back(8); ihdr.push_back(2); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  FILE* f = std::fopen(path, "wb");
  if (!f) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  return (std::fclose(f) == 0 && ok) ? MCPT_OK : MCPT_ERR_INVALID_ARG;
}

// checkpoint file (mcpt.h): magic, 6 int32 (W, rows, pass_count, next_pass, tag bytes, H),
// uint64 row-list hash, tag, floats.  H = 0 / hash = 0: no target identity (mcpt_checkpoint_write).
// "MCPTCKP1" files (round 3: 5 int32, no identity) are still read.
static const char kCkptMagic[8] = {'M', 'C', 'P', 'T', 'C', 'K', 'P', '2'};
static const char kCkptMagicV1[8] = {'M', 'C', 'P', 'T', 'C', 'K', 'P', '1'};

namespace mcpt {
namespace host {
// The file is written to a temporary name unique to this process and thread, flushed to the
// device (fsync) and renamed over `path`: a killed process or a host crash leaves either the
// previous checkpoint or the new one, and two writers never share a temporary file.
int checkpoint_write_ex(const char* path, const float* rgb, int W, int rows, int pass_count, int next_pass,
                        const char* tag, int H, unsigned long long rows_hash) {
  if (!path || !rgb || W <= 0 || rows <= 0 || pass_count < 0 || H < 0) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  const size_t tag_len = tag ? std::strlen(tag) : 0;
  if (tag_len >= MCPT_CHECKPOINT_TAG_MAX) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  char suffix[64];
  std::snprintf(suffix, sizeof(suffix), ".tmp.%ld.%zx", (long)getpid(), std::hash<std::thread::id>()(std::this_thread::get_id()));
  const std::string tmp = std::string(path) + suffix;
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  const int32_t hdr[6] = {W, rows, pass_count, next_pass, (int32_t)tag_len, H};
  const uint64_t hash = rows_hash;
  const size_t n = (size_t)W * rows * 3;
  bool ok = std::fwrite(kCkptMagic, 1, 8, f) == 8 && std::fwrite(hdr, sizeof(int32_t), 6, f) == 6 &&
            std::fwrite(&hash, sizeof(hash), 1, f) == 1 && std::fwrite(tag ? tag : "", 1, tag_len, f) == tag_len &&
            std::fwrite(rgb, sizeof(float), n, f) == n;
  ok = ok && std::fflush(f) == 0 && fsync(fileno(f)) == 0;
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path) != 0) {
    std::remove(tmp.c_str());
    return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  }
  // the rename itself reaches the device with the directory's metadata
  std::string dir(path);
  const size_t slash = dir.find_last_of('/');
  dir = slash == std::string::npos ? std::string(".") : (slash == 0 ? std::string("/") : dir.substr(0, slash));
  const int dfd = open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (dfd >= 0) {
    (void)fsync(dfd);
    (void)close(dfd);
  }
  return MCPT_OK;
}

int checkpoint_read_ex(const char* path, float* rgb_out, long long capacity, int* W, int* rows, int* pass_count,
                       int* next_pass, char* tag_out, int* H, unsigned long long* rows_hash) {
  if (!path) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  FILE* f = std::fopen(path, "rb");
  if (!f) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  char magic[8];
  int32_t hdr[6] = {0, 0, 0, 0, 0, 0};
  uint64_t hash = 0;
  char tag[MCPT_CHECKPOINT_TAG_MAX];
  bool ok = std::fread(magic, 1, 8, f) == 8;
  const bool v2 = ok && std::memcmp(magic, kCkptMagic, 8) == 0;
  ok = ok && (v2 || std::memcmp(magic, kCkptMagicV1, 8) == 0) &&
       std::fread(hdr, sizeof(int32_t), v2 ? 6 : 5, f) == (size_t)(v2 ? 6 : 5) &&
       (!v2 || std::fread(&hash, sizeof(hash), 1, f) == 1) && hdr[0] > 0 && hdr[1] > 0 && hdr[2] >= 0 &&
       hdr[4] >= 0 && hdr[4] < MCPT_CHECKPOINT_TAG_MAX && hdr[5] >= 0 &&
       std::fread(tag, 1, (size_t)hdr[4], f) == (size_t)hdr[4];
  if (ok && rgb_out) {
    const size_t n = (size_t)hdr[0] * hdr[1] * 3;
    ok = capacity >= 0 && n <= (size_t)capacity && std::fread(rgb_out, sizeof(float), n, f) == n;
  }
  std::fclose(f);
  if (!ok) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  tag[hdr[4]] = '\0';
  if (W) *W = hdr[0];
  if (rows) *rows = hdr[1];
  if (pass_count) *pass_count = hdr[2];
  if (next_pass) *next_pass = hdr[3];
  if (tag_out) std::memcpy(tag_out, tag, (size_t)hdr[4] + 1);
  if (H) *H = hdr[5];
  if (rows_hash) *rows_hash = hash;
  return MCPT_OK;
}
}  // namespace host
}  // namespace mcpt

int mcpt_checkpoint_write(const char* path, const float* rgb, int W, int rows, int pass_count, int next_pass,
                          const char* tag) {
  return mcpt::host::checkpoint_write_ex(path, rgb, W, rows, pass_count, next_pass, tag, 0, 0);
}

int mcpt_checkpoint_read(const char* path, float* rgb_out, long long capacity, int* W, int* rows, int* pass_count,
                         int* next_pass, char* tag_out) {
  return mcpt::host::checkpoint_read_ex(path, rgb_out, capacity, W, rows, pass_count, next_pass, tag_out, nullptr,
                                        nullptr);
}

int mcpt_transfo_translate(float x, float y, float z, float* out16) {
  if (!out16) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  mcpt::host::transfo_translate(x, y, z, out16);
  return MCPT_OK;
}
int mcpt_transfo_scale(float x, float y, float z, float* out16) {
  if (!out16) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  mcpt::host::transfo_scale(x, y, z, out16);
  return MCPT_OK;
}
int mcpt_transfo_rotate(int axis, float degrees, float* out16) {
  if (!out16 || axis < 0 || axis > 2) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  mcpt::host::transfo_rotate(axis, degrees, out16);
  return MCPT_OK;
}
int mcpt_mat4_mul(const float* a16, const float* b16, float* out16) {
  if (!a16 || !b16 || !out16) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  mcpt::host::mat4_mul(a16, b16, out16);
  return MCPT_OK;
}

}  // extern "C"
