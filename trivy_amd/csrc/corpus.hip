// corpus.hip — seeded synthetic source-tree generator (bench/test utility,
// not part of the scan path).  Implements the SURVEY.md §8(d) text model:
// lines of 20–160 bytes of identifiers (45 %), CamelCase/UPPER words (10 %),
// numbers (10 %), punctuation (15 %), base64-ish blobs (10 %) and blanks
// (10 %), with builtin-rule secrets planted at line starts at a given density
// (secrets per byte) and 20 % one-char-short decoys of fixed-length tokens.
//
// Every 4 KiB chunk of every file is generated independently from
// hash(seed, file, chunk), so the same bytes come out of the device kernel
// (bench corpora of tens of GB) and of the host function (oracle spot checks).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "trivy_secret_gpu.h"

namespace {

constexpr uint32_t kGenChunk = 4096;

struct Rng {
  uint64_t s;
  __host__ __device__ uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  __host__ __device__ uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
  __host__ __device__ double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

__host__ __device__ inline uint64_t mix(uint64_t a, uint64_t b) {
  Rng r{a * 0xD1B54A32D192ED03ull ^ b};
  return r.next();
}

#define LOWER "abcdefghijklmnopqrstuvwxyz"
#define UPPER "ABCDEFGHIJKLMNOPQRSTUVWXYZ"
#define DIGIT "0123456789"

struct Tpl {
  const char* prefix;   // literal text before the token
  const char* charset;  // token alphabet
  uint8_t len;          // token length
  const char* suffix;   // literal text after the token
  uint8_t fixed;        // one-char-short decoy is a guaranteed non-match
  uint8_t group_off;    // expected location = [line + group_off, line + group_off + group_len)
  uint8_t group_len;    //   (0 = whole prefix+token+suffix)
};

// Templates (line-start instances); rule ids in the comments.
constexpr Tpl kTpl[] = {
    {"AWS_ACCESS_KEY_ID=AKIA", UPPER DIGIT, 16, "", 1, 18, 20},                   // aws-access-key-id (group)
    {"aws_secret_access_key = \"", UPPER LOWER DIGIT "/+=", 40, "\"", 0, 25, 40},  // aws-secret-access-key (group)
    {"ghp_", UPPER LOWER DIGIT, 36, "", 1, 0, 0},                                // github-pat
    {"gho_", UPPER LOWER DIGIT, 36, "", 1, 0, 0},                                // github-oauth
    {"glpat-", UPPER LOWER DIGIT, 20, "", 1, 0, 0},                              // gitlab-pat
    {"hf_", UPPER LOWER DIGIT, 39, "", 1, 0, 0},                                 // hugging-face-access-token
    {"xoxb-", UPPER LOWER DIGIT, 30, "", 0, 0, 0},                               // slack-access-token
    {"sk_live_", LOWER DIGIT, 24, "", 0, 0, 0},                                  // stripe-secret-token
    {"SG.", UPPER LOWER DIGIT "_-.", 66, "", 1, 0, 0},                           // sendgrid-api-token
    {"\"npm_", LOWER DIGIT, 36, "\"", 1, 0, 0},                                  // npm-access-token
    {"facebook_secret = \"", "0123456789abcdef", 32, "\"", 1, 19, 32},           // facebook-token (group)
    {"SK", "0123456789abcdef", 32, "", 1, 0, 0},                                 // twilio-api-key
    {"shpat_", "0123456789abcdef", 32, "", 1, 0, 0},                             // shopify-token
    {"AGE-SECRET-KEY-1", "QPZRY9X8GF2TVDW0S3JN54KHCE6MUA7L", 58, "", 1, 0, 0},   // age-secret-key
    {"rubygems_", "0123456789abcdef", 48, "", 1, 0, 0},                          // rubygems-api-token
    {"pul-", "0123456789abcdef", 40, "", 1, 0, 0},                               // pulumi-api-token
};
constexpr int kNumTpl = (int)(sizeof(kTpl) / sizeof(kTpl[0]));
constexpr char kPunct[] = "=:\"'{}[](),.;";
constexpr char kB64[] = UPPER LOWER DIGIT "+/=";
constexpr char kId[] = LOWER "_";
constexpr int kMaxPlantsPerChunk = 8;

__host__ __device__ inline uint32_t slen(const char* s) {
  uint32_t n = 0;
  while (s[n]) ++n;
  return n;
}

struct Plant {
  uint32_t file;
  uint32_t tpl;
  uint64_t start, end;  // expected location (file-relative)
  uint32_t decoy;
  uint32_t pad;
};

// Generate chunk `c` of file `f` (length n) into out[0..n); planted secrets
// are reported into plants[0..*np) (at most kMaxPlantsPerChunk).
__host__ __device__ inline void gen_chunk(uint64_t seed, uint32_t f, uint32_t c, uint32_t n, uint8_t* out,
                                          double density, Plant* plants, int* np, uint64_t chunk_off) {
  Rng r{mix(seed ^ 0x5EC2E7ull, ((uint64_t)f << 20) ^ c)};
  uint32_t pos = 0, line_pos = 0;
  uint32_t line_target = 20 + r.below(141);
  const double p_line = density * 90.0;
  *np = 0;
  while (pos < n) {
    if (line_pos == 0 && (pos > 0 || c == 0) && n - pos > 200 && *np < kMaxPlantsPerChunk && r.unit() < p_line) {
      const uint32_t ti = r.below((uint32_t)kNumTpl);
      const Tpl& t = kTpl[ti];
      const bool decoy = t.fixed && r.unit() < 0.2;
      const uint32_t tl = t.len - (decoy ? 1 : 0);
      const uint32_t start = pos;
      for (const char* q = t.prefix; *q; ++q) out[pos++] = (uint8_t)*q;
      const uint32_t cs = slen(t.charset);
      for (uint32_t k = 0; k < tl; ++k) out[pos++] = (uint8_t)t.charset[r.below(cs)];
      for (const char* q = t.suffix; *q; ++q) out[pos++] = (uint8_t)*q;
      const uint32_t end = pos;
      out[pos++] = '\n';
      Plant& p = plants[(*np)++];
      p.file = f;
      p.tpl = ti;
      p.decoy = decoy;
      p.pad = 0;
      p.start = chunk_off + (t.group_len ? start + t.group_off : start);
      p.end = chunk_off + (t.group_len ? start + t.group_off + t.group_len : end);
      line_target = 20 + r.below(141);
      continue;
    }
    uint32_t k = r.below(100);
    uint32_t len;
    if (k < 45) {
      len = 2 + r.below(13);
      for (uint32_t i = 0; i < len && pos < n; ++i) out[pos++] = (uint8_t)kId[r.below(27)];
    } else if (k < 55) {
      len = 2 + r.below(7);
      const bool camel = r.below(2);
      for (uint32_t i = 0; i < len && pos < n; ++i) {
        const uint32_t ch = r.below(26);
        out[pos++] = (uint8_t)((camel && i > 0) ? 'a' + ch : 'A' + ch);
      }
    } else if (k < 65) {
      len = 1 + r.below(8);
      for (uint32_t i = 0; i < len && pos < n; ++i) out[pos++] = (uint8_t)('0' + r.below(10));
    } else if (k < 80) {
      len = 1;
      out[pos++] = (uint8_t)kPunct[r.below(13)];
    } else if (k < 90) {
      len = 16 + r.below(65);
      for (uint32_t i = 0; i < len && pos < n; ++i) out[pos++] = (uint8_t)kB64[r.below(65)];
    } else {
      len = 1;
      out[pos++] = (uint8_t)(r.below(4) ? ' ' : '\t');
    }
    line_pos += len;
    if (pos < n) {
      if (line_pos >= line_target) {
        out[pos++] = '\n';
        line_pos = 0;
        line_target = 20 + r.below(141);
      } else {
        out[pos++] = ' ';
        line_pos++;
      }
    }
  }
}

// One thread per 4 KiB chunk; chunk_id[i] = (file << 24) | chunk index.
__global__ __launch_bounds__(256) void k_gen(uint8_t* data, const uint64_t* off, const uint64_t* chunk_id,
                                             uint64_t n_chunks, uint64_t seed, double density, Plant* plants,
                                             unsigned long long* nplants, uint64_t plant_cap) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_chunks) return;
  const uint32_t f = (uint32_t)(chunk_id[i] >> 24);
  const uint32_t c = (uint32_t)(chunk_id[i] & 0xFFFFFF);
  const uint64_t fstart = off[f], flen = off[f + 1] - off[f] - 1;  // NUL separator after each file
  const uint64_t cstart = (uint64_t)c * kGenChunk;
  const uint32_t n = (uint32_t)((flen - cstart) < kGenChunk ? (flen - cstart) : kGenChunk);
  Plant local[kMaxPlantsPerChunk];
  int np = 0;
  gen_chunk(seed, f, c, n, data + fstart + cstart, density, local, &np, cstart);
  for (int k = 0; k < np; ++k) {
    unsigned long long idx = atomicAdd(nplants, 1ull);
    if (idx < plant_cap) plants[idx] = local[k];
  }
}

constexpr const char* kExt[] = {"cfg", "env", "ini", "jsx", "tsx", "cpp", "php", "xml", "txt", "yml"};

__global__ void k_paths(uint8_t* paths, uint64_t* path_off, uint64_t n_files, uint64_t seed) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_files) return;
  path_off[i] = i * 31;
  if (i == n_files) return;
  // "srcNN/pkgNNN/fileNNNNNNNNNN.ext" (31 bytes), no allow-path substrings
  Rng r{mix(seed ^ 0x9A71ull, i)};
  char buf[32];
  int p = 0;
  auto put = [&](const char* s) { while (*s) buf[p++] = *s++; };
  auto num = [&](uint64_t v, int w) {
    for (int k = w - 1; k >= 0; --k) { buf[p + k] = (char)('0' + v % 10); v /= 10; }
    p += w;
  };
  put("src"); num(r.below(100), 2); put("/pkg"); num(r.below(1000), 3); put("/file"); num(i, 10);
  buf[p++] = '.';
  put(kExt[r.below(10)]);  // 3-letter extensions keep every path 31 bytes
  for (int k = 0; k < 31; ++k) paths[i * 31 + k] = (uint8_t)buf[k];
}

}  // namespace

extern "C" {

// Fill a device corpus: d_data (capacity >= offsets[n]), d_offsets[n+1] and
// d_chunk_file (one (file << 24 | chunk) entry per 4 KiB chunk) precomputed by the host;
// paths are 31 bytes each.  Planted secrets are recorded into d_plants.
int tsg_gen_corpus_device(uint8_t* d_data, const uint64_t* d_offsets, const uint64_t* d_chunk_file,
                          uint64_t n_chunks, uint8_t* d_paths, uint64_t* d_path_offsets, uint64_t n_files,
                          uint64_t seed, double density, void* d_plants, uint64_t plant_cap,
                          unsigned long long* d_nplants) {
  if (n_chunks)
    hipLaunchKernelGGL(k_gen, dim3((uint32_t)((n_chunks + 255) / 256)), dim3(256), 0, 0, d_data, d_offsets,
                       d_chunk_file, n_chunks, seed, density, (Plant*)d_plants, d_nplants, plant_cap);
  hipLaunchKernelGGL(k_paths, dim3((uint32_t)((n_files + 1 + 255) / 256)), dim3(256), 0, 0, d_paths,
                     d_path_offsets, n_files, seed);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TSG_ERR_DEVICE;
  return TSG_OK;
}

// Host twin of the device generator: bytes of file f (length n).
int tsg_gen_file(uint64_t seed, uint32_t f, uint64_t n, double density, uint8_t* out) {
  Plant local[kMaxPlantsPerChunk];
  int np = 0;
  for (uint64_t c = 0; c * kGenChunk < n; ++c) {
    const uint64_t cs = c * kGenChunk;
    const uint32_t len = (uint32_t)((n - cs) < kGenChunk ? (n - cs) : kGenChunk);
    gen_chunk(seed, f, (uint32_t)c, len, out + cs, density, local, &np, cs);
  }
  return TSG_OK;
}

size_t tsg_gen_plant_record_size(void) { return sizeof(Plant); }
uint32_t tsg_gen_chunk_bytes(void) { return kGenChunk; }

}  // extern "C"
