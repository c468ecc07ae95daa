// corpus.hip — seeded synthetic source-tree generator (bench/test utility,
// not part of the scan path).  Implements the SURVEY.md §8(d) text model:
// lines of 20–160 bytes of identifiers (45 %), CamelCase/UPPER words (10 %),
// numbers (10 %), punctuation (15 %), base64-ish blobs (10 %) and blanks
// (10 %), with an instance of EVERY builtin rule (builtin-rules.go:95-823,
// one template per rule, chosen uniformly) planted at line starts at a given
// density (secrets per byte); 20 % of plants are decoys: one character short
// (templates whose shortened segment can no longer match) or carrying
// "EXAMPLE" inside the match (dropped by the builtin allow rule `(?i)example`,
// builtin-allow-rules.go:13).  0.1 % of files carry a few non-ASCII runes
// (é, K U+212A, ſ U+017F, İ U+0130), some of them as rule instances whose
// k/s letters are spelled K/ſ (Go's (?i) simple folding matches them; the
// expectation of those comes from the oracle, not from the generator).
//
// Every 4 KiB chunk of every file is generated independently from
// hash(seed, file, chunk), so the same bytes come out of the device kernel
// (bench corpora of tens of GB) and of the host function (oracle spot checks).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "tsg_corpus.h"
#include "trivy_secret_gpu.h"  // TSG_OK / TSG_ERR_DEVICE

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

// Template language (one line per builtin rule, in builtin-rules.go order):
//   {N:c} / {N-M:c}  N (or N..M) random characters of charset c (kCharsets)
//   (a|b|c)          one literal alternative, uniformly
//   < ... >          the Location the rule reports (secret group); absent =>
//                    the whole instance
//   !{..}            the segment a one-char-short decoy shortens (marks the
//                    template "fixed": the short instance can never match)
//   ^{..}            the segment an EXAMPLE decoy overwrites (first 7 chars)
struct Tpl {
  const char* rule;
  const char* pat;
};

constexpr Tpl kTpl[] = {
    {"aws-access-key-id", "AWS_ACCESS_KEY_ID=<(AKIA|AGPA|AIDA|AROA|AIPA|ANPA|ANVA|ASIA)^!{16:U}>"},
    {"aws-secret-access-key", "aws_secret_access_key = \"<^!{40:B}>\""},
    {"github-pat", "ghp_^!{36:A}"},
    {"github-oauth", "gho_^!{36:A}"},
    {"github-app-token", "(ghu|ghs)_^!{36:A}"},
    {"github-refresh-token", "ghr_^!{76:A}"},
    {"github-fine-grained-pat", "github_pat_^{22:A}_!{59:A}"},
    {"gitlab-pat", "glpat-^!{20:x}"},
    {"hugging-face-access-token", "hf_^!{39:A}"},
    {"private-key", "-----BEGIN (RSA|EC|OPENSSH) PRIVATE KEY-----<\n^{64:B}\n{16-64:B}\n>-----END RSA PRIVATE KEY-----"},
    {"shopify-token", "shp(ss|at|ca|pa)_!{32:h}"},
    {"slack-access-token", "xox(b|a|p|r|s)-^{10-48:A}"},
    {"stripe-publishable-token", "pk_(test|live)_^{10-32:l}"},
    {"stripe-secret-token", "sk_(test|live)_^{10-32:l}"},
    {"pypi-upload-token", "pypi-AgEIcHlwaS5vcmc^{50-200:x}"},
    {"gcp-service-account", "  <\"type\": \"service_account\">,"},
    {"heroku-api-key", " heroku_api_key = \"<{8:H}-{4:H}-{4:H}-{4:H}-!{12:H}>\""},
    {"slack-web-hook", "https://hooks.slack.com/services/^{44-48:S}"},
    {"twilio-api-key", "SK!{32:h}"},
    {"age-secret-key", "AGE-SECRET-KEY-1!{58:Q}"},
    {"facebook-token", "facebook_secret = \"<!{32:h}>\""},
    {"twitter-token", "twitter_api_secret: \"<{35-44:h}>\""},
    {"adobe-client-id", "adobe_client_id = \"<!{32:h}>\""},
    {"adobe-client-secret", "p8e-^!{32:l}"},
    {"alibaba-access-key-id", "<LTAI^!{20:l}>"},
    {"alibaba-secret-key", "alibaba_secret = '<^!{30:l}>'"},
    {"asana-client-id", "asana_client_id = \"<!{16:d}>\""},
    {"asana-client-secret", "asana_secret = \"<^!{32:l}>\""},
    {"atlassian-api-token", "atlassian_token := \"<^!{24:l}>\""},
    {"bitbucket-client-id", "bitbucket_key = \"<^!{32:l}>\""},
    {"bitbucket-client-secret", "bitbucket_secret = \"<^!{64:w}>\""},
    {"beamer-api-token", "beamer_token = \"<b_^!{44:y}>\""},
    {"clojars-api-token", "CLOJARS_^!{60:l}"},
    {"contentful-delivery-api-token", "contentful_token = \"<^!{43:y}>\""},
    {"databricks-api-token", "dapi!{32:g}"},
    {"discord-api-token", "discord_token = \"<!{64:g}>\""},
    {"discord-client-id", "discord_id = \"<!{18:d}>\""},
    {"discord-client-secret", "discord_secret = \"<^!{32:y}>\""},
    {"doppler-api-token", "token: <\"dp.pt.^!{43:l}\">"},
    {"dropbox-api-secret", "<dropbox_key = \"^!{15:l}\">"},
    {"dropbox-short-lived-api-token", "<dropbox_token = \"sl.^!{135:y}\">"},
    {"dropbox-long-lived-api-token", "<dropbox_token = \"^{11:l}AAAAAAAAAA!{43:y}\">"},
    {"duffel-api-token", "key: <\"duffel_(test|live)_^!{43:w}\">"},
    {"dynatrace-api-token", "<\"dt0c01.^{24:l}.!{64:l}\">"},
    {"easypost-api-token", "<\"EZAK^!{54:l}\">"},
    {"fastly-api-token", "fastly_api = \"<^!{32:y}>\""},
    {"finicity-client-secret", "finicity_secret = \"<^!{20:l}>\""},
    {"finicity-api-token", "finicity_token = \"<!{32:h}>\""},
    {"flutterwave-public-key", "FLW(PUB|SEC)K_TEST-!{32:g}-X"},
    {"flutterwave-enc-key", "FLWSECK_TEST!{12:g}"},
    {"frameio-api-token", "fio-u-^!{64:y}"},
    {"gocardless-api-token", "<\"live_^!{40:y}\">"},
    {"grafana-api-token", "<\"eyJrIjoi^{72-92:y}\">"},
    {"hashicorp-tf-api-token", "<\"^{14:l}.atlasv1.{60-70:y}\">"},
    {"hubspot-api-token", "hubspot_key = \"<{8:g}-{4:g}-{4:g}-{4:g}-!{12:g}>\""},
    {"intercom-api-token", "intercom_token = \"<^!{60:m}>\""},
    {"intercom-client-secret", "intercom_secret = \"<{8:g}-{4:g}-{4:g}-{4:g}-!{12:g}>\""},
    {"ionic-api-token", "<ionic_key = \"ion_^!{42:l}\">"},
    {"jwt-token", "jwt = <ey^{20:A}.ey{25:v}.{30:v}>"},
    {"linear-api-token", "lin_api_^!{40:l}"},
    {"linear-client-secret", "linear_secret = \"<!{32:h}>\""},
    {"lob-api-key", "lob_key = \"<(live|test)_!{35:h}>\""},
    {"lob-pub-api-key", "lob_pub = \"<(test|live)_pub_!{31:h}>\""},
    {"mailchimp-api-key", "mailchimp_key = \"<{32:h}-us20>\""},
    {"mailgun-token", "mailgun_key = \"<key-!{32:h}>\""},
    {"mailgun-signing-key", "mailgun_signing = \"<{32:g}-{8:g}-!{8:g}>\""},
    {"mapbox-api-token", "pk.^{60:l}.!{22:l}"},
    {"messagebird-api-token", "messagebird_key = \"<^!{25:l}>\""},
    {"messagebird-client-id", "messagebird_id = \"<{8:g}-{4:g}-{4:g}-{4:g}-!{12:g}>\""},
    {"new-relic-user-api-key", "<\"NRAK-^!{27:U}\">"},
    {"new-relic-user-api-id", "newrelic_id = \"<^!{64:U}>\""},
    {"new-relic-browser-api-token", "<\"NRJS-!{19:h}\">"},
    {"npm-access-token", "<\"npm_^!{36:l}\">"},
    {"planetscale-password", "pscale_pw_^!{43:p}"},
    {"planetscale-api-token", "pscale_tkn_^!{43:p}"},
    {"postman-api-token", "PMAK-{24:h}-!{34:h}"},
    {"pulumi-api-token", "pul-!{40:h}"},
    {"rubygems-api-token", "rubygems_!{48:h}"},
    {"sendgrid-api-token", "SG.^!{66:p}"},
    {"sendinblue-api-token", "xkeysib-{64:h}-^!{16:l}"},
    {"shippo-api-token", "shippo_(live|test)_!{40:h}"},
    {"linkedin-client-secret", "linkedin_secret = \"<^!{16:a}>\""},
    {"linkedin-client-id", "linkedin_id = \"<^!{14:l}>\""},
    {"twitch-api-token", "twitch_token = \"<^!{30:l}>\""},
    {"typeform-api-token", "typeform_key = <tfp_^!{59:q}>"},
    {"dockerconfig-secret", "  .dockerconfigjson: <ey^{30:B}>"},
};
constexpr int kNumTpl = (int)(sizeof(kTpl) / sizeof(kTpl[0]));
static_assert(kNumTpl == 86, "one template per builtin rule");

#define LOWER "abcdefghijklmnopqrstuvwxyz"
#define UPPER "ABCDEFGHIJKLMNOPQRSTUVWXYZ"
#define DIGIT "0123456789"

__host__ __device__ inline const char* charset(char c) {
  switch (c) {
    case 'U': return UPPER DIGIT;
    case 'A': return UPPER LOWER DIGIT;
    case 'B': return UPPER LOWER DIGIT "/+=";
    case 'h': return "0123456789abcdef";
    case 'H': return "0123456789ABCDEF";
    case 'l': return LOWER DIGIT;
    case 'a': return LOWER;
    case 'g': return "abcdefgh0123456789";
    case 'd': return DIGIT;
    case 'x': return UPPER LOWER DIGIT "-_";
    case 'y': return LOWER DIGIT "-_=";
    case 'w': return LOWER DIGIT "_-";
    case 'm': return LOWER DIGIT "=_";
    case 'p': return LOWER DIGIT "-_.";
    case 'q': return LOWER DIGIT "-_.=";
    case 'S': return UPPER LOWER DIGIT "+/";
    case 'v': return UPPER LOWER DIGIT "/_-";
    case 'Q': return "QPZRY9X8GF2TVDW0S3JN54KHCE6MUA7L";
    default: return "x";
  }
}

constexpr uint8_t kRunes[4][3] = {{0xC3, 0xA9, 0}, {0xE2, 0x84, 0xAA}, {0xC5, 0xBF, 0}, {0xC4, 0xB0, 0}};
constexpr char kPunct[] = "=:\"'{}[](),.;";
constexpr char kB64[] = UPPER LOWER DIGIT "+/=";
constexpr char kId[] = LOWER "_";
constexpr int kMaxPlantsPerChunk = 8;
constexpr uint32_t kTplMaxBytes = 600;  // longest instance (private-key, pypi), fold spellings included

__host__ __device__ inline uint32_t slen(const char* s) {
  uint32_t n = 0;
  while (s[n]) ++n;
  return n;
}

enum PlantKind : uint32_t { PLANT_REAL = 0, PLANT_SHORT = 1, PLANT_EXAMPLE = 2, PLANT_FOLD = 3 };

struct Plant {
  uint32_t file;
  uint32_t tpl;
  uint64_t start, end;  // expected location (file-relative)
  uint32_t decoy;       // PlantKind
  uint32_t pad;
};

__host__ __device__ inline uint32_t parse_num(const char*& q) {
  uint32_t v = 0;
  while (*q >= '0' && *q <= '9') v = v * 10 + (uint32_t)(*q++ - '0');
  return v;
}

__host__ __device__ inline bool tpl_fixed(const char* p) {
  for (; *p; ++p)
    if (*p == '!') return true;
  return false;
}

__host__ __device__ inline bool tpl_example(const char* p) {
  for (; *p; ++p)
    if (*p == '^') return true;
  return false;
}

// Write one instance of template t at out (room for kTplMaxBytes).  kind:
// PLANT_SHORT shortens the '!' segment by one, PLANT_EXAMPLE writes
// "EXAMPLE" over the start of the '^' segment, PLANT_FOLD spells the
// literal k/s letters as K (E2 84 AA) / ſ (C5 BF) at random.  Returns the
// instance length; *ls/*le = the expected location.
__host__ __device__ inline uint32_t write_instance(const Tpl& t, Rng& r, uint32_t kind, uint8_t* out, uint32_t* ls,
                                                   uint32_t* le) {
  uint32_t pos = 0;
  *ls = 0xFFFFFFFFu;
  *le = 0xFFFFFFFFu;
  bool short_next = false, example_next = false;
  for (const char* q = t.pat; *q;) {
    const char ch = *q;
    if (ch == '<') { *ls = pos; ++q; continue; }
    if (ch == '>') { *le = pos; ++q; continue; }
    if (ch == '!') { short_next = true; ++q; continue; }
    if (ch == '^') { example_next = true; ++q; continue; }
    if (ch == '(') {  // literal alternatives
      const char* a = q + 1;
      uint32_t nalt = 1;
      for (const char* z = a; *z != ')'; ++z) nalt += *z == '|';
      uint32_t pick = r.below(nalt);
      const char* z = a;
      while (pick) { if (*z++ == '|') --pick; }
      for (; *z != '|' && *z != ')'; ++z) out[pos++] = (uint8_t)*z;
      while (*q != ')') ++q;
      ++q;
      continue;
    }
    if (ch == '{') {
      ++q;
      uint32_t lo = parse_num(q), hi = lo;
      if (*q == '-') { ++q; hi = parse_num(q); }
      const char* cs = charset(q[1]);  // q -> ':'
      q += 3;                           // ":c}"
      uint32_t n = lo + (hi > lo ? r.below(hi - lo + 1) : 0);
      if (short_next && kind == PLANT_SHORT) --n;
      const uint32_t ncs = slen(cs);
      const uint32_t s0 = pos;
      for (uint32_t k = 0; k < n; ++k) out[pos++] = (uint8_t)cs[r.below(ncs)];
      if (example_next && kind == PLANT_EXAMPLE && n >= 7) {
        const char* ex = "EXAMPLE";
        for (int k = 0; k < 7; ++k) out[s0 + k] = (uint8_t)ex[k];
      }
      short_next = example_next = false;
      continue;
    }
    uint8_t c = (uint8_t)ch;
    if (kind == PLANT_FOLD && (c == 'k' || c == 'K') && r.below(2)) {
      out[pos++] = 0xE2; out[pos++] = 0x84; out[pos++] = 0xAA;
    } else if (kind == PLANT_FOLD && (c == 's' || c == 'S') && r.below(2)) {
      out[pos++] = 0xC5; out[pos++] = 0xBF;
    } else {
      out[pos++] = c;
    }
    ++q;
  }
  if (*ls == 0xFFFFFFFFu) { *ls = 0; *le = pos; }
  return pos;
}

__host__ __device__ inline bool file_nonascii(uint64_t seed, uint32_t f) {
  return (mix(seed ^ 0x0A5C11ull, f) >> 11) % 1000 == 0;  // 0.1 % of files
}

// Generate chunk `c` of file `f` (chunk length n, file length flen) into
// out[0..n); planted secrets are reported into plants[0..*np) (at most
// kMaxPlantsPerChunk).
__host__ __device__ inline void gen_chunk(uint64_t seed, uint32_t f, uint32_t c, uint32_t n, uint64_t flen, uint8_t* out,
                                          double density, Plant* plants, int* np, uint64_t chunk_off) {
  Rng r{mix(seed ^ 0x5EC2E7ull, ((uint64_t)f << 20) ^ c)};
  uint32_t pos = 0, line_pos = 0;
  uint32_t line_target = 20 + r.below(141);
  const double p_line = density * 90.0;
  // non-ASCII files: ~3 runes per file, a quarter of them as K/ſ-spelled rule instances
  uint32_t runes_left = 0;
  if (file_nonascii(seed, f)) {
    const double nch = (double)((flen + kGenChunk - 1) / kGenChunk);
    if (r.unit() < (nch <= 3.0 ? 1.0 : 3.0 / nch)) runes_left = nch <= 3.0 ? 2 : 1;
  }
  *np = 0;
  while (pos < n) {
    const bool line_start = line_pos == 0 && (pos > 0 || c == 0);
    if (line_start && n - pos > kTplMaxBytes + 2 && *np < kMaxPlantsPerChunk && r.unit() < p_line) {
      const uint32_t ti = r.below((uint32_t)kNumTpl);
      const Tpl& t = kTpl[ti];
      uint32_t kind = PLANT_REAL;
      if (r.unit() < 0.2) {
        const bool fx = tpl_fixed(t.pat), ex = tpl_example(t.pat);
        if (fx && ex) kind = r.below(2) ? PLANT_SHORT : PLANT_EXAMPLE;
        else if (fx) kind = PLANT_SHORT;
        else if (ex) kind = PLANT_EXAMPLE;
      }
      uint32_t ls, le;
      const uint32_t len = write_instance(t, r, kind, out + pos, &ls, &le);
      Plant& p = plants[(*np)++];
      p.file = f;
      p.tpl = ti;
      p.decoy = kind;
      p.pad = 0;
      p.start = chunk_off + pos + ls;
      p.end = chunk_off + pos + le;
      pos += len;
      out[pos++] = '\n';
      line_target = 20 + r.below(141);
      continue;
    }
    if (runes_left && line_start && n - pos > kTplMaxBytes + 2 && r.unit() < 1.0 / 30.0) {
      --runes_left;
      if (r.below(4) == 0 && *np < kMaxPlantsPerChunk) {  // K/ſ-spelled instance: expectation from the oracle
        const uint32_t ti = r.below((uint32_t)kNumTpl);
        uint32_t ls, le;
        const uint32_t len = write_instance(kTpl[ti], r, PLANT_FOLD, out + pos, &ls, &le);
        Plant& p = plants[(*np)++];
        p.file = f;
        p.tpl = ti;
        p.decoy = PLANT_FOLD;
        p.pad = 0;
        p.start = chunk_off + pos + ls;
        p.end = chunk_off + pos + le;
        pos += len;
        out[pos++] = '\n';
        continue;
      }
      // one rune inside a word: é, K, ſ or İ
      const uint32_t k = r.below(4);
      for (uint32_t i = 0; i < 3 && kRunes[k][i]; ++i) out[pos++] = kRunes[k][i];
      const uint32_t wl = 2 + r.below(6);
      for (uint32_t i = 0; i < wl; ++i) out[pos++] = (uint8_t)kId[r.below(27)];
      out[pos++] = ' ';
      line_pos = wl + 4;
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
  gen_chunk(seed, f, c, n, flen, data + fstart + cstart, density, local, &np, cstart);
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

// Host twin of the device generator: bytes of file f (length n); its plants
// (up to plant_cap records) into plants / *n_plants when plants is non-null.
int tsg_gen_file_plants(uint64_t seed, uint32_t f, uint64_t n, double density, uint8_t* out, void* plants,
                        size_t plant_cap, size_t* n_plants) {
  Plant local[kMaxPlantsPerChunk];
  int np = 0;
  size_t total = 0;
  for (uint64_t c = 0; c * kGenChunk < n; ++c) {
    const uint64_t cs = c * kGenChunk;
    const uint32_t len = (uint32_t)((n - cs) < kGenChunk ? (n - cs) : kGenChunk);
    gen_chunk(seed, f, (uint32_t)c, len, n, out + cs, density, local, &np, cs);
    for (int k = 0; k < np; ++k, ++total)
      if (plants && total < plant_cap) ((Plant*)plants)[total] = local[k];
  }
  if (n_plants) *n_plants = total;
  return TSG_OK;
}

int tsg_gen_file(uint64_t seed, uint32_t f, uint64_t n, double density, uint8_t* out) {
  return tsg_gen_file_plants(seed, f, n, density, out, nullptr, 0, nullptr);
}

int tsg_gen_file_nonascii(uint64_t seed, uint32_t f) { return file_nonascii(seed, f) ? 1 : 0; }

size_t tsg_gen_template_count(void) { return (size_t)kNumTpl; }
const char* tsg_gen_template_rule(size_t i) { return i < (size_t)kNumTpl ? kTpl[i].rule : nullptr; }
size_t tsg_gen_plant_record_size(void) { return sizeof(Plant); }
uint32_t tsg_gen_chunk_bytes(void) { return kGenChunk; }

}  // extern "C"
