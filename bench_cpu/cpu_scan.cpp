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
#include <vector>

#include "engine.h"
#include "pikevm.h"

namespace {

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

std::atomic<uint64_t> g_sink{0};

struct Blocks {
  const std::vector<int>* regexes;
  bool done = false;
  std::vector<Loc> locs;
  bool match(const Ctx& C, Vm& vm, const uint8_t* t, uint32_t n, Loc l) {
    if (!done) {
      done = true;
      for (int r : *regexes) find_all(C, vm, r, t, n, [&](uint32_t a, uint32_t b) { locs.push_back({a, b}); });
    }
    for (auto& b : locs)
      if (b.s <= l.s && l.e <= b.e) return true;
    return false;
  }
};

// toFinding's findLocation (scanner.go:481-537): line numbers and the match line
uint64_t finding_cost(const uint8_t* t, uint32_t n, Loc l) {
  uint64_t start_line = 1 + std::count(t, t + l.s, (uint8_t)'\n');
  uint64_t end_line = start_line + std::count(t + l.s, t + l.e, (uint8_t)'\n');
  const uint8_t* ls = t + l.s;
  while (ls > t && ls[-1] != '\n') --ls;
  const uint8_t* le = (const uint8_t*)memchr(t + l.e, '\n', n - l.e);
  return start_line ^ (end_line << 20) ^ (uint64_t)((le ? le : t + n) - ls);
}

uint64_t scan_file(const Ctx& C, Vm& vm, std::string& lower, std::vector<uint8_t>& censored, const uint8_t* t,
                   uint32_t n, const char* path) {
  const tsg_ruleset* rs = C.rs;
  const uint32_t plen = (uint32_t)strlen(path);
  for (int r : rs->global_allow_path)
    if (match_string(C, vm, r, (const uint8_t*)path, plen)) return 0;
  Blocks global{&rs->global_exclude};
  bool lowered = false, copied = false;
  uint64_t found = 0, sink = 0;
  for (const auto& rule : rs->rules) {
    if (rule.path >= 0 && !match_string(C, vm, rule.path, (const uint8_t*)path, plen)) continue;
    bool allowed = false;
    for (int r : rule.allow_path) allowed = allowed || match_string(C, vm, r, (const uint8_t*)path, plen);
    if (allowed) continue;
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
      if (!any) continue;
    }
    if (rule.regex < 0) continue;
    const gre::Prog& prog = *C.rx[rule.regex].prog;
    std::vector<Loc> locs;
    std::vector<uint32_t> slots;
    if (!rule.group_name.empty())
      for (size_t g = 0; g < prog.cap_names.size(); ++g)
        if (prog.cap_names[g] == rule.group_name) slots.push_back((uint32_t)g);
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
      for (uint32_t g : slots)
        if (caps[2 * g] >= 0) locs.push_back({(uint32_t)caps[2 * g], (uint32_t)caps[2 * g + 1]});
    });
    if (locs.empty()) continue;
    Blocks local{&rule.exclude};
    for (auto& l : locs) {
      if (global.match(C, vm, t, n, l) || local.match(C, vm, t, n, l)) continue;
      if (!copied) {
        censored.assign(t, t + n);
        copied = true;
      }
      memset(censored.data() + l.s, '*', l.e - l.s);
      sink += finding_cost(censored.data(), n, l);
      ++found;
    }
  }
  g_sink.fetch_xor(sink, std::memory_order_relaxed);  // keeps the findLocation work observable
  return found;
}

}  // namespace

extern "C" {

// Scan n_files files (content data[off[i] .. off[i+1]-1), a NUL after each, as
// in the GPU batch layout) with `threads` threads.  Writes per-file finding
// counts (may be null), the total, and the scan's wall seconds.
int tsgb_cpu_scan(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* off, size_t n_files,
                  const char* const* paths, int threads, uint32_t* per_file, uint64_t* total, double* seconds) {
  if (!rs || !data || !off || !paths || !total || !seconds || threads < 1) return TSG_ERR_INVALID_ARG;
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
  std::atomic<size_t> next{0};
  std::atomic<uint64_t> sum{0};
  auto t0 = std::chrono::steady_clock::now();
  auto work = [&]() {
    Vm vm(C.max_inst, C.max_cap);
    std::string lower;
    std::vector<uint8_t> censored;
    uint64_t mine = 0;
    for (size_t f; (f = next.fetch_add(1)) < n_files;) {
      const uint32_t len = (uint32_t)(off[f + 1] - 1 - off[f]);
      const uint64_t k = scan_file(C, vm, lower, censored, data + off[f], len, paths[f]);
      if (per_file) per_file[f] = (uint32_t)k;
      mine += k;
    }
    sum += mine;
  };
  std::vector<std::thread> ts;
  for (int i = 1; i < threads; ++i) {
    try {
      ts.emplace_back(work);
    } catch (...) {
      break;  // fewer threads: the remaining ones take the files
    }
  }
  work();
  for (auto& th : ts) th.join();
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *total = sum.load();
  return TSG_OK;
}

}  // extern "C"
