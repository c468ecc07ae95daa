// cpu_scan.cpp — bench-only CPU baseline: the reference's Scanner.Scan
// (pkg/fanal/secret/scanner.go:371-452) restated in C++ over this repo's own
// host regexp VM (gre::vm_search / vm_captures, the Go-semantics Pike VM of
// pikevm.h), multi-threaded over files.  NOT the product path (that is
// libtrivy_secret_gpu.so on the GPU) and NOT the oracle: bench.py times it as
// `cpu_baseline` kind "cpp-restatement" — a C++ restatement, not Go.
//
// Per file, in the reference's order:
//   global AllowPath (scanner.go:375)           -> MatchString of each global allow-path regex
//   global exclude blocks (:389, :255-270)      -> FindAllIndex, lazily on the first location
//   per rule: MatchPath / AllowPath (:391-399), MatchKeywords (:169-181),
//             FindLocations (:97-143) with AllowLocation (:145-148),
//             rule exclude blocks, censoring copy (:425-433), toFinding's line
//             numbers (:464-537)
// One deliberate speed-up over Go: the content is lowered once per file
// (Go lowers it once per keyword per rule, scanner.go:175); the keyword
// result is the same.  Regex searches start at Go's literal prefix
// (regexp.go onepass / machine prefix skip), as Go's matcher does.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "engine.h"
#include "pikevm.h"

namespace {

// ---- finding digests (full-size parity: bench.py compares these per file) ----
// XXH64 (Collet's published algorithm, seed 0; tests/test_cpu_baseline.py
// checks it against the python xxhash module).
constexpr uint64_t kP1 = 11400714785074694791ull, kP2 = 14029467366897019727ull, kP3 = 1609587929392839161ull,
                   kP4 = 9650029242287828579ull, kP5 = 2870177450012600261ull;
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline uint64_t xround(uint64_t acc, uint64_t in) { return rotl64(acc + in * kP2, 31) * kP1; }
inline uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * kP1 + kP4; }

uint64_t tsgb_xxh64(const uint8_t* p, size_t n) {
  const uint8_t* const end = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = kP1 + kP2, v2 = kP2, v3 = 0, v4 = 0 - kP1;
    for (const uint8_t* lim = end - 32; p <= lim; p += 32) {
      v1 = xround(v1, rd64(p));
      v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16));
      v4 = xround(v4, rd64(p + 24));
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(xmerge(xmerge(xmerge(h, v1), v2), v3), v4);
  } else {
    h = kP5;
  }
  h += (uint64_t)n;
  for (; p + 8 <= end; p += 8) h = rotl64(h ^ xround(0, rd64(p)), 27) * kP1 + kP4;
  if (p + 4 <= end) {
    h = rotl64(h ^ ((uint64_t)rd32(p) * kP1), 23) * kP2 + kP3;
    p += 4;
  }
  for (; p < end; ++p) h = rotl64(h ^ ((uint64_t)*p * kP5), 11) * kP1;
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  return h;
}

struct tsgb_line_key {
  uint32_t number;       // types.Line.Number
  uint8_t flags;         // 1 IsCause, 2 FirstCause, 4 LastCause
  uint64_t content_hash; // tsgb_xxh64 of Content
};

// One finding: XXH64 of rule u32 | start u64 | end u64 | StartLine u32 |
// EndLine u32 | xxh64(Match) u64 | n_lines u32 | per line: Number u32,
// flags u8, xxh64(Content) u64 (little-endian, packed).
uint64_t tsgb_finding_hash(uint32_t rule, uint64_t start, uint64_t end, uint32_t sl, uint32_t el, uint64_t mh,
                           const tsgb_line_key* lines, size_t n_lines) {
  std::vector<uint8_t> b(40 + 13 * n_lines);
  uint8_t* w = b.data();
  auto put = [&](const void* v, size_t k) {
    memcpy(w, v, k);
    w += k;
  };
  const uint32_t nl32 = (uint32_t)n_lines;
  put(&rule, 4), put(&start, 8), put(&end, 8), put(&sl, 4), put(&el, 4), put(&mh, 8), put(&nl32, 4);
  for (size_t q = 0; q < n_lines; ++q) put(&lines[q].number, 4), put(&lines[q].flags, 1), put(&lines[q].content_hash, 8);
  return tsgb_xxh64(b.data(), (size_t)(w - b.data()));
}

struct Vm {
  std::vector<uint16_t> sp0, sp1, d0, d1, stk;
  std::vector<uint32_t> s0, s1;
  std::vector<int32_t> c0, c1, cur, cst;
  gre::VmScratch sc{};
  Vm(size_t ninst, size_t ncap)
      : sp0(ninst), sp1(ninst), d0(ninst), d1(ninst), stk(ninst + 1), s0(ninst), s1(ninst),
        c0(ninst * ncap), c1(ninst * ncap), cur(ncap), cst(2 * ninst + 2) {
    sc.sparse[0] = sp0.data();
    sc.sparse[1] = sp1.data();
    sc.dense[0] = d0.data();
    sc.dense[1] = d1.data();
    sc.start[0] = s0.data();
    sc.start[1] = s1.data();
    sc.stack = stk.data();
    sc.caps[0] = c0.data();
    sc.caps[1] = c1.data();
    sc.cur = cur.data();
    sc.capstack = cst.data();
  }
};

gre::ProgView view(const gre::Prog& p) {
  return gre::ProgView{p.inst.data(), p.classes.data(), p.ranges.data(), (uint32_t)p.inst.size(), p.start,
                       (uint32_t)p.ncap, p.nvis};
}

// Go's Prog.Prefix: the case-sensitive literal every match starts with.
std::string literal_prefix(const gre::Prog& p) {
  auto skip = [&](uint32_t pc) {
    while (pc && (p.inst[pc].op == gre::I_NOP || p.inst[pc].op == gre::I_CAP)) pc = p.inst[pc].out;
    return pc;
  };
  std::string out;
  uint32_t pc = skip(p.start);
  while (pc && p.inst[pc].op == gre::I_RUNE1 && p.inst[pc].arg < 0x80) {
    out.push_back((char)p.inst[pc].arg);
    pc = skip(p.inst[pc].out);
  }
  return out;
}

struct Regex {
  const gre::Prog* prog = nullptr;
  gre::ProgView pv{};
  std::string prefix;
};

struct Ctx {
  const tsg_ruleset* rs;
  std::vector<Regex> rx;
  size_t max_inst = 1, max_cap = 2;
};

bool match_string(const Ctx& C, Vm& vm, int r, const uint8_t* s, uint32_t n) {
  uint32_t ms, me;
  return gre::vm_search(C.rx[r].pv, s, n, 0, n, true, vm.sc, &ms, &me);
}

// Go regexp.go allMatches (FindAllIndex), each search started at the next
// occurrence of the literal prefix.
template <class F>
void find_all(const Ctx& C, Vm& vm, int r, const uint8_t* t, uint32_t n, F&& on_match) {
  const Regex& R = C.rx[r];
  int64_t prev_end = -1;
  uint32_t pos = 0;
  while (pos <= n) {
    uint32_t from = pos;
    if (!R.prefix.empty()) {
      const void* h = memmem(t + pos, n - pos, R.prefix.data(), R.prefix.size());
      if (!h) break;
      from = (uint32_t)((const uint8_t*)h - t);
    }
    uint32_t ms, me;
    if (!gre::vm_search(R.pv, t, n, from, n, false, vm.sc, &ms, &me)) break;
    bool accept = true;
    if (me == pos) {
      if ((int64_t)ms == prev_end) accept = false;
      uint32_t w;
      gre::decode_rune(t, n, pos, &w);
      pos = w > 0 ? pos + w : n + 1;
    } else {
      pos = me;
    }
    prev_end = me;
    if (accept) on_match(ms, me);
  }
}

// bytes.ToLower for ASCII keywords: ASCII lowered, U+0130 -> 'i', U+212A ->
// 'k', every other non-ASCII rune (or invalid byte) -> one 0x80 byte.
void to_lower_kw(const uint8_t* s, uint32_t n, std::string& out) {
  out.clear();
  out.reserve(n);
  for (uint32_t i = 0; i < n;) {
    const uint8_t c = s[i];
    if (c < 0x80) {
      out.push_back((char)(c >= 'A' && c <= 'Z' ? c + 32 : c));
      ++i;
      continue;
    }
    uint32_t w;
    const int r = gre::decode_rune(s, n, i, &w);
    out.push_back(r == 0x130 ? 'i' : r == 0x212A ? 'k' : (char)0x80);
    i += w ? w : 1;
  }
}

struct Loc {
  uint32_t s, e;
};

struct Blocks {
  const std::vector<int>* regexes;
  bool done = false;
  std::vector<Loc> locs;
  void ensure(const Ctx& C, Vm& vm, const uint8_t* t, uint32_t n) {
    if (!done) {
      done = true;
      for (int r : *regexes) find_all(C, vm, r, t, n, [&](uint32_t a, uint32_t b) { locs.push_back({a, b}); });
    }
  }
  bool match(const Ctx& C, Vm& vm, const uint8_t* t, uint32_t n, Loc l) {
    ensure(C, vm, t, n);
    for (auto& b : locs)
      if (b.s <= l.s && l.e <= b.e) return true;
    return false;
  }
};

struct Kept {
  uint32_t rule, s, e;
};

// Per-thread scratch of one file's findings.
struct FileScratch {
  std::string lower;
  std::vector<uint8_t> censored;
  std::vector<Kept> kept;
  std::vector<uint32_t> nl;                        // newline positions of the censored content
  std::unordered_map<uint32_t, uint64_t> memo;  // line index -> content hash (Code lines shared by findings)
};

// toFinding / findLocation (scanner.go:464-537) on the fully censored content
// c[0..n), hashed as tsgb_finding_hash: the rule index, the location, StartLine,
// EndLine, the Match window and every Code line (Number, flags, Content).
uint64_t finding_digest(FileScratch& F, const uint8_t* c, uint32_t n, const Kept& k) {
  const std::vector<uint32_t>& nl = F.nl;
  const uint32_t sl = (uint32_t)(std::lower_bound(nl.begin(), nl.end(), k.s) - nl.begin());  // bytes.Count(content[:start])
  const uint32_t el = (uint32_t)(std::lower_bound(nl.begin(), nl.end(), k.e) - nl.begin());  // + Count(content[start:end])
  uint64_t ls = sl == 0 ? 0 : (uint64_t)nl[sl - 1] + 1;        // LastIndex(content[:start], "\n") + 1
  uint64_t le = sl < nl.size() ? (uint64_t)nl[sl] : (uint64_t)n;  // Index(content[start:], "\n") + start
  if (le - ls > 100) {
    ls = k.s >= 30 ? k.s - 30 : 0;
    le = std::min<uint64_t>((uint64_t)k.e + 20, n);
  }
  const uint64_t mh = tsgb_xxh64(c + ls, (size_t)(le - ls));
  const uint32_t n_split = (uint32_t)nl.size() + 1;  // len(bytes.Split(content, "\n"))
  const uint32_t cs = sl >= 2 ? sl - 2 : 0;
  const uint32_t ce = std::min(el + 2, n_split);
  std::vector<tsgb_line_key> lines;
  lines.reserve(ce - cs);
  bool first = false;
  for (uint32_t i = cs; i < ce; ++i) {
    auto it = F.memo.find(i);
    uint64_t h;
    if (it != F.memo.end()) {
      h = it->second;
    } else {
      const uint64_t a = i == 0 ? 0 : (uint64_t)nl[i - 1] + 1;
      const uint64_t b = i < nl.size() ? (uint64_t)nl[i] : (uint64_t)n;
      h = tsgb_xxh64(c + a, (size_t)(b - a));
      F.memo.emplace(i, h);
    }
    const bool cause = i >= sl && i <= el;
    tsgb_line_key lk{};
    lk.number = i + 1;
    lk.flags = (uint8_t)((cause ? 1 : 0) | (cause && !first ? 2 : 0));
    lk.content_hash = h;
    first = first || cause;
    lines.push_back(lk);
  }
  for (size_t q = lines.size(); q-- > 0;)
    if (lines[q].flags & 1) {
      lines[q].flags |= 4;  // LastCause
      break;
    }
  return tsgb_finding_hash(k.rule, k.s, k.e, sl + 1, el + 1, mh, lines.data(), lines.size());
}

// One file's view shared by the rules of its scan.
struct FileView {
  const uint8_t* t;
  uint32_t n;
  const char* path;
  uint32_t plen;
};

// One rule of Scan's loop (scanner.go:388-434): path gates, MatchKeywords on
// the lowered content (lowered once per file, `lower` filled on first need),
// FindLocations with AllowLocation, exclude blocks; kept locations appended.
void scan_rule(const Ctx& C, Vm& vm, const FileView& v, uint32_t ri, std::string& lower, bool& lowered,
               Blocks& global, std::vector<Loc>& locs, std::vector<Kept>& kept) {
  const tsg_ruleset* rs = C.rs;
  const auto& rule = rs->rules[ri];
  const uint8_t* t = v.t;
  const uint32_t n = v.n;
  if (rule.path >= 0 && !match_string(C, vm, rule.path, (const uint8_t*)v.path, v.plen)) return;
  for (int r : rule.allow_path)
    if (match_string(C, vm, r, (const uint8_t*)v.path, v.plen)) return;
  if (!rule.keywords.empty()) {
    if (!lowered) {
      to_lower_kw(t, n, lower);
      lowered = true;
    }
    bool any = false;
    for (auto& kw : rule.keywords)
      if (kw.empty() || memmem(lower.data(), lower.size(), kw.data(), kw.size())) {
        any = true;
        break;
      }
    if (!any) return;
  }
  if (rule.regex < 0) return;
  const gre::Prog& prog = *C.rx[rule.regex].prog;
  locs.clear();
  uint32_t slots[tsg::kMaxCap];
  uint32_t n_slots = 0;
  if (!rule.group_name.empty())
    for (size_t g = 0; g < prog.cap_names.size() && n_slots < tsg::kMaxCap; ++g)
      if (prog.cap_names[g] == rule.group_name) slots[n_slots++] = (uint32_t)g;
  int32_t caps[2 * tsg::kMaxCap];
  find_all(C, vm, rule.regex, t, n, [&](uint32_t ms, uint32_t me) {
    for (int r : rs->global_allow_regex)  // AllowLocation: global then rule allow regexes
      if (match_string(C, vm, r, t + ms, me - ms)) return;
    for (int r : rule.allow_regex)
      if (match_string(C, vm, r, t + ms, me - ms)) return;
    if (rule.group_name.empty()) {
      locs.push_back({ms, me});
      return;
    }
    gre::vm_captures(C.rx[rule.regex].pv, t, n, ms, vm.sc, caps);
    for (uint32_t q = 0; q < n_slots; ++q)
      if (caps[2 * slots[q]] >= 0) locs.push_back({(uint32_t)caps[2 * slots[q]], (uint32_t)caps[2 * slots[q] + 1]});
  });
  if (locs.empty()) return;
  Blocks local{&rule.exclude};
  for (auto& l : locs) {
    if (global.match(C, vm, t, n, l) || local.match(C, vm, t, n, l)) continue;
    kept.push_back({ri, l.s, l.e});
  }
}

// censorLocation over every kept location, then toFinding on the result;
// returns the count, *digest = the sum of the findings' tsgb_finding_hash
// (order-free: Scan's (RuleID, Match) ties are).
uint32_t finish_file(FileScratch& F, const FileView& v, uint64_t* digest) {
  *digest = 0;
  if (F.kept.empty()) return 0;
  const uint32_t n = v.n;
  F.censored.assign(v.t, v.t + n);
  for (auto& k : F.kept) memset(F.censored.data() + k.s, '*', k.e - k.s);
  const uint8_t* c = F.censored.data();
  F.nl.clear();
  for (const uint8_t* p = c; (p = (const uint8_t*)memchr(p, '\n', c + n - p)) != nullptr; ++p)
    F.nl.push_back((uint32_t)(p - c));
  F.memo.clear();
  uint64_t sum = 0;
  for (auto& k : F.kept) sum += finding_digest(F, c, n, k);
  *digest = sum;
  return (uint32_t)F.kept.size();
}

bool path_allowed(const Ctx& C, Vm& vm, const FileView& v) {  // Global AllowPath (scanner.go:375)
  for (int r : C.rs->global_allow_path)
    if (match_string(C, vm, r, (const uint8_t*)v.path, v.plen)) return true;
  return false;
}

// Scanner.Scan of one file on one thread.
uint32_t scan_file(const Ctx& C, Vm& vm, FileScratch& F, const FileView& v, uint64_t* digest) {
  *digest = 0;
  F.kept.clear();
  if (path_allowed(C, vm, v)) return 0;
  Blocks global{&C.rs->global_exclude};
  bool lowered = false;
  std::vector<Loc> locs;
  for (uint32_t ri = 0; ri < C.rs->rules.size(); ++ri) scan_rule(C, vm, v, ri, F.lower, lowered, global, locs, F.kept);
  return finish_file(F, v, digest);
}

}  // namespace

extern "C" {

uint64_t tsgb_xxh64_bytes(const uint8_t* p, size_t n) { return tsgb_xxh64(p, n); }

// Scan n_files files (content data[off[i] .. off[i+1]-1), a NUL after each, as
// in the GPU batch layout) with `threads` threads (see big_file_bytes below).  Writes per-file finding
// counts and digests (either may be null: tsgb_finding_hash summed over the
// file's findings), the total, and the scan's wall seconds.
int tsgb_cpu_scan(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* off, size_t n_files,
                  const char* const* paths, int threads, uint64_t big_file_bytes, uint32_t* per_file,
                  uint64_t* per_file_digest, uint64_t* total, double* seconds) {
  if (!rs || !data || !off || !paths || !total || !seconds || threads < 1) return TSG_ERR_INVALID_ARG;
  for (size_t f = 0; f < n_files; ++f)
    if (off[f + 1] - off[f] - 1 >= (1ull << 32)) return TSG_ERR_UNSUPPORTED;  // 32-bit positions
  Ctx C;
  C.rs = rs;
  for (auto& r : rs->regexes) {
    Regex x;
    x.prog = &r.c.prog;
    x.pv = view(r.c.prog);
    x.prefix = literal_prefix(r.c.prog);
    C.rx.push_back(x);
    C.max_inst = std::max(C.max_inst, r.c.prog.inst.size() + 1);
    C.max_cap = std::max(C.max_cap, (size_t)r.c.prog.ncap);
  }
  // Files of big_file_bytes or more (0: 4 MiB) run one at a time with the
  // rules spread over the threads (each rule's FindAll is independent; the
  // kept locations are merged in rule order before censoring), the rest one
  // file per thread.
  const uint64_t kBigFile = big_file_bytes ? big_file_bytes : (4u << 20);
  std::vector<size_t> big;
  for (size_t f = 0; f < n_files; ++f)
    if (off[f + 1] - 1 - off[f] >= kBigFile) big.push_back(f);
  std::atomic<size_t> next{0};
  std::atomic<uint64_t> sum{0};
  auto view_of = [&](size_t f) {
    return FileView{data + off[f], (uint32_t)(off[f + 1] - 1 - off[f]), paths[f], (uint32_t)strlen(paths[f])};
  };
  auto t0 = std::chrono::steady_clock::now();
  auto run_threads = [&](auto&& work) {
    std::vector<std::thread> ts;
    for (int i = 1; i < threads; ++i) {
      try {
        ts.emplace_back(work);
      } catch (...) {
        break;  // fewer threads: the remaining ones take the work
      }
    }
    work();
    for (auto& th : ts) th.join();
  };
  run_threads([&]() {
    Vm vm(C.max_inst, C.max_cap);
    FileScratch F;
    uint64_t mine = 0;
    for (size_t f; (f = next.fetch_add(1)) < n_files;) {
      const FileView v = view_of(f);
      if (v.n >= kBigFile) continue;
      uint64_t d = 0;
      const uint32_t k = scan_file(C, vm, F, v, &d);
      if (per_file) per_file[f] = k;
      if (per_file_digest) per_file_digest[f] = d;
      mine += k;
    }
    sum += mine;
  });
  for (size_t f : big) {
    const FileView v = view_of(f);
    FileScratch F;
    uint64_t d = 0;
    uint32_t k = 0;
    Vm vm0(C.max_inst, C.max_cap);
    if (!path_allowed(C, vm0, v)) {
      Blocks global{&rs->global_exclude};
      global.ensure(C, vm0, v.t, v.n);  // read-only from here on
      to_lower_kw(v.t, v.n, F.lower);
      const size_t nr = rs->rules.size();
      std::vector<std::vector<Kept>> per_rule(nr);
      std::atomic<size_t> next_rule{0};
      run_threads([&]() {
        Vm vm(C.max_inst, C.max_cap);
        bool lowered = true;
        std::vector<Loc> locs;
        for (size_t ri; (ri = next_rule.fetch_add(1)) < nr;)
          scan_rule(C, vm, v, (uint32_t)ri, F.lower, lowered, global, locs, per_rule[ri]);
      });
      for (auto& pr : per_rule) F.kept.insert(F.kept.end(), pr.begin(), pr.end());
      k = finish_file(F, v, &d);
    }
    if (per_file) per_file[f] = k;
    if (per_file_digest) per_file_digest[f] = d;
    sum += k;
  }
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *total = sum.load();
  return TSG_OK;
}

// The same digests from an engine result, read through the drop-in ABI as a
// caller sees it: `findings` = tsg_result_findings of the loaded engine
// library (passed in so this bench library does not link the product), files
// [file0, file0 + n_files) of `result`.  Code line hashes are memoised by
// their arena pointer (a line shared by many findings is stored once).
typedef size_t (*tsgb_findings_fn)(const tsg_result*, size_t, const tsg_finding**);
int tsgb_result_digest(void* findings, const tsg_result* result, size_t file0, size_t n_files, uint32_t* count,
                       uint64_t* digest) {
  if (!findings || !result || !count || !digest) return TSG_ERR_INVALID_ARG;
  auto fn = (tsgb_findings_fn)findings;
  std::unordered_map<const char*, std::pair<size_t, uint64_t>> memo;
  std::vector<tsgb_line_key> lines;
  for (size_t i = 0; i < n_files; ++i) {
    const tsg_finding* fs = nullptr;
    const size_t k = fn(result, file0 + i, &fs);
    uint64_t sum = 0;
    for (size_t j = 0; j < k; ++j) {
      const tsg_finding& f = fs[j];
      lines.clear();
      for (size_t q = 0; q < f.n_lines; ++q) {
        const tsg_line& L = f.lines[q];
        auto it = memo.find(L.content);
        uint64_t h;
        if (it != memo.end() && it->second.first == L.content_len) {
          h = it->second.second;
        } else {
          h = tsgb_xxh64((const uint8_t*)L.content, L.content_len);
          memo[L.content] = {L.content_len, h};
        }
        tsgb_line_key lk{};
        lk.number = L.number;
        lk.flags = (uint8_t)((L.is_cause ? 1 : 0) | (L.first_cause ? 2 : 0) | (L.last_cause ? 4 : 0));
        lk.content_hash = h;
        lines.push_back(lk);
      }
      sum += tsgb_finding_hash(f.rule, f.start, f.end, f.start_line, f.end_line,
                               tsgb_xxh64((const uint8_t*)f.match, f.match_len), lines.data(), lines.size());
    }
    count[i] = (uint32_t)k;
    digest[i] = sum;
  }
  return TSG_OK;
}

// One finding's hash from its fields (the test computes the oracle's side
// through this too, so the serialisation is defined once): Match and each
// Code line's Content arrive as their tsgb_xxh64.
uint64_t tsgb_finding_hash_c(uint32_t rule, uint64_t start, uint64_t end, uint32_t start_line, uint32_t end_line,
                             uint64_t match_hash, const uint32_t* numbers, const uint8_t* flags,
                             const uint64_t* content_hashes, size_t n_lines) {
  std::vector<tsgb_line_key> lines(n_lines);
  for (size_t q = 0; q < n_lines; ++q) lines[q] = {numbers[q], flags[q], content_hashes[q]};
  return tsgb_finding_hash(rule, start, end, start_line, end_line, match_hash, lines.data(), n_lines);
}

// configs[0] through the caller-filled staging (bench --staged): every file
// reserved in order through `add` (the product library's tsg_staging_add,
// passed in as a pointer: this library does not link it), then the contents
// copied into their slots by `threads` threads over equal byte shares -- as
// the tagged build's analyzer workers io.ReadFull into theirs.  Returns the
// files staged (n unless the staging filled up).
typedef int (*tsgb_stage_add_fn)(void* st, const char* path, uint64_t len, uint8_t** dst);
size_t tsgb_stage_files(void* st, tsgb_stage_add_fn add, const uint8_t* data, const uint64_t* off,
                        const uint64_t* len, const char* const* paths, size_t n, int threads) {
  std::vector<uint8_t*> dst(n);
  size_t k = 0;
  for (; k < n; ++k)
    if (add(st, paths[k], len[k], &dst[k]) != TSG_OK) break;
  uint64_t total = 0;
  for (size_t i = 0; i < k; ++i) total += len[i];
  threads = std::max(1, threads);
  std::vector<std::thread> pool;
  std::atomic<size_t> next{0};
  const uint64_t share = total / threads + 1;
  // file ranges of about `share` bytes each, claimed in order
  std::vector<size_t> cut{0};
  uint64_t acc = 0;
  for (size_t i = 0; i < k; ++i) {
    acc += len[i];
    if (acc >= share * cut.size()) cut.push_back(i + 1);
  }
  if (cut.back() != k) cut.push_back(k);
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (size_t c; (c = next.fetch_add(1)) + 1 < cut.size();)
        for (size_t i = cut[c]; i < cut[c + 1]; ++i) memcpy(dst[i], data + off[i], len[i]);
    });
  for (auto& t : pool) t.join();
  return k;
}

}  // extern "C"
