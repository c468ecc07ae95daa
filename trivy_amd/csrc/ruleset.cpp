// Host rule compiler: turns the Rule / AllowRule / ExcludeBlock model of
// pkg/fanal/secret/scanner.go:84-95,191-221 into the engine's compiled form:
// Go-RE2 programs (gre.cpp), anchor literals, and one Aho-Corasick automaton
// over every keyword (MatchKeywords, scanner.go:169-181) and anchor literal.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>

#include "engine.h"
#include "gre_lower_table.h"
#include "pikevm.h"

namespace {
thread_local std::string g_last_error;
std::atomic<uint64_t> g_ruleset_ids{1};

void set_err(char* err, size_t errlen, const std::string& msg) {
  g_last_error = msg;
  if (err && errlen) {
    size_t n = std::min(errlen - 1, msg.size());
    memcpy(err, msg.data(), n);
    err[n] = '\0';
  }
}

std::string ascii_lower(const std::string& s) {
  std::string o = s;
  for (auto& c : o)
    if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
  return o;
}

// strings.ToLower (scanner.go:174-176, keywords): Go's unicode.ToLower per
// rune (gre_lower_table.h); false for invalid UTF-8 (RuneError substitution
// in a keyword is outside this engine's coverage).
bool go_lower_utf8(const std::string& in, std::string* out) {
  out->clear();
  const uint8_t* b = (const uint8_t*)in.data();
  const uint32_t n = (uint32_t)in.size();
  for (uint32_t i = 0; i < n;) {
    uint32_t w = 0;
    int r = gre::decode_rune(b, n, i, &w);
    if (r == 0xFFFD && !(w == 3 && b[i] == 0xEF && b[i + 1] == 0xBF && b[i + 2] == 0xBD)) return false;
    uint32_t lr = (uint32_t)r;
    if (lr < 0x80) {
      if (lr >= 'A' && lr <= 'Z') lr += 32;
    } else {
      int lo = 0, hi = kLowerMapLen;
      while (lo < hi) {
        const int m = (lo + hi) / 2;
        if (kLowerMap[m][0] < lr) lo = m + 1;
        else hi = m;
      }
      if (lo < kLowerMapLen && kLowerMap[lo][0] == lr) lr = kLowerMap[lo][1];
    }
    char e[4];
    int k = 0;
    if (lr < 0x80) e[k++] = (char)lr;
    else if (lr < 0x800) { e[k++] = (char)(0xC0 | (lr >> 6)); e[k++] = (char)(0x80 | (lr & 0x3F)); }
    else if (lr < 0x10000) { e[k++] = (char)(0xE0 | (lr >> 12)); e[k++] = (char)(0x80 | ((lr >> 6) & 0x3F)); e[k++] = (char)(0x80 | (lr & 0x3F)); }
    else { e[k++] = (char)(0xF0 | (lr >> 18)); e[k++] = (char)(0x80 | ((lr >> 12) & 0x3F)); e[k++] = (char)(0x80 | ((lr >> 6) & 0x3F)); e[k++] = (char)(0x80 | (lr & 0x3F)); }
    out->append(e, k);
    i += w;
  }
  return true;
}

bool is_ascii(const std::string& s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}
}  // namespace

namespace tsg {
void set_last_error(const std::string& m) { g_last_error = m; }

// Aho-Corasick over the lowercased patterns (truncated to `depth` bytes).
static bool build_ac_depth(tsg_ruleset* rs, int depth, std::string* err) {
  AcHost& ac = rs->ac;
  ac = AcHost{};
  ac.depth = (uint32_t)depth;
  // byte classes: every byte that appears in a (lowercased) pattern gets a
  // class; 'A'-'Z' share the class of their lowercase letter.
  int cmap[256];
  for (int b = 0; b < 256; ++b) cmap[b] = 0;
  int ncls = 1;
  for (auto& p : rs->patterns) {
    size_t L = std::min<size_t>(p.lower.size(), (size_t)depth);
    for (size_t k = 0; k < L; ++k) {
      unsigned char c = p.lower[k];
      if (c == 0) {
        *err = "NUL bytes in keywords/literals are outside this engine's coverage (NUL separates files)";
        return false;
      }
      if (!cmap[c]) cmap[c] = ncls++;
    }
  }
  for (int b = 'A'; b <= 'Z'; ++b) cmap[b] = cmap[b + 32];
  for (int b = 0; b < 256; ++b) ac.cls[b] = (uint8_t)cmap[b];
  if (ncls > 255) {
    *err = "too many byte classes";
    return false;
  }
  // trie
  std::vector<std::vector<int>> go;  // [state][class] -> state or -1
  std::vector<std::vector<uint16_t>> term;
  go.push_back(std::vector<int>(ncls, -1));
  term.emplace_back();
  for (size_t pi = 0; pi < rs->patterns.size(); ++pi) {
    auto& p = rs->patterns[pi];
    size_t L = std::min<size_t>(p.lower.size(), (size_t)depth);
    int s = 0;
    for (size_t k = 0; k < L; ++k) {
      int c = cmap[(unsigned char)p.lower[k]];
      if (go[s][c] < 0) {
        go[s][c] = (int)go.size();
        go.push_back(std::vector<int>(ncls, -1));
        term.emplace_back();
      }
      s = go[s][c];
    }
    term[s].push_back((uint16_t)pi);
  }
  int S = (int)go.size();
  if (S >= 32768) {
    *err = "keyword automaton too large";
    return false;
  }
  std::vector<int> fail(S, 0);
  std::vector<std::vector<uint16_t>> outs(S);
  std::deque<int> q;
  for (int c = 0; c < ncls; ++c) {
    if (go[0][c] < 0) {
      go[0][c] = 0;
    } else {
      fail[go[0][c]] = 0;
      q.push_back(go[0][c]);
    }
  }
  outs[0] = term[0];
  std::vector<int> order;
  while (!q.empty()) {
    int s = q.front();
    q.pop_front();
    order.push_back(s);
    outs[s] = term[s];
    for (auto x : outs[fail[s]]) outs[s].push_back(x);
    for (int c = 0; c < ncls; ++c) {
      int t = go[s][c];
      if (t >= 0) {
        fail[t] = go[fail[s]][c];
        q.push_back(t);
      } else {
        go[s][c] = go[fail[s]][c];
      }
    }
  }
  // renumber: states without outputs first (root stays 0), output states
  // last, each part in breadth-first order, so shallow states (where text
  // keeps the automaton) have the smallest ids: k_scan_generic keeps the
  // first rows of a table too large for LDS in LDS
  {
    std::vector<int> bfs;
    bfs.push_back(0);
    bfs.insert(bfs.end(), order.begin(), order.end());
    std::vector<int> perm(S), inv;
    for (int st : bfs)
      if (outs[st].empty()) { perm[st] = (int)inv.size(); inv.push_back(st); }
    for (int st : bfs)
      if (!outs[st].empty()) { perm[st] = (int)inv.size(); inv.push_back(st); }
    std::vector<std::vector<int>> go2(S);
    std::vector<std::vector<uint16_t>> outs2(S);
    for (int n = 0; n < S; ++n) {
      go2[n] = go[inv[n]];
      for (auto& t : go2[n]) t = perm[t];
      outs2[n] = outs[inv[n]];
    }
    go.swap(go2);
    outs.swap(outs2);
    // failure links in the new numbering (k_scan_big's sparse cold rows)
    ac.fail.assign(S, 0);
    for (int n = 0; n < S; ++n) ac.fail[n] = (uint16_t)perm[fail[inv[n]]];
  }
  ac.nstates = (uint32_t)S;
  ac.nclasses = (uint32_t)ncls;
  ac.delta.assign((size_t)S * ncls, 0);
  for (int s = 0; s < S; ++s)
    for (int c = 0; c < ncls; ++c) {
      int t = go[s][c];
      uint16_t v = (uint16_t)t;
      if (!outs[t].empty()) v |= 0x8000;
      ac.delta[(size_t)s * ncls + c] = v;
    }
  ac.out_off.assign(S + 1, 0);
  ac.out_pat.clear();
  for (int s = 0; s < S; ++s) {
    ac.out_off[s] = (uint32_t)ac.out_pat.size();
    for (auto x : outs[s]) ac.out_pat.push_back(x);
  }
  ac.out_off[S] = (uint32_t)ac.out_pat.size();
  return true;
}

// k_scan_fast's automaton: a DFA over the 64 fold columns (engine.hip fold6:
// both letter cases share a column; control bytes, bytes >= 0x80 and a few
// rare ASCII bytes alias other columns, so every reported pattern is
// confirmed on the real bytes by k_report) for the patterns truncated to
// `depth`, each anchor-only literal followed by plan[pattern] of its required
// column sets (PatternHost::ext_cols).  Built by subset construction
// over items (pattern, columns matched); a state's outputs are the patterns
// completed on entering it, and output states are numbered last so the scan
// detects an output with one max() per byte.  Entry = next row's index, so a
// step reads the u16 at e * kFastRowBytes + 2 * col.  Only for all-ASCII pattern sets whose rows
// fit 16-bit entries and the LDS image (the fold-special sequences are found
// by k_fold_special instead).
static bool build_fast(tsg_ruleset* rs, int depth, const std::vector<uint8_t>& plan) {
  AcHost& ac = rs->ac;
  ac.fast.clear();
  ac.fast_out_off.clear();
  ac.fast_out_pat.clear();
  ac.fast_states = 0;
  ac.fast_out_entry = 0;
  ac.fast_ev_entry = 0;
  ac.fast_kw.clear();
  ac.fast_kw_map.clear();
  ac.fast_ext.assign(rs->patterns.size(), 0);
  ac.fast_pair.clear();
  for (auto& p : rs->patterns)
    if (!p.special)
      for (unsigned char c : p.lower)
        if (c >= 0x80) return false;
  const size_t max_rows = kFastMaxRows;
  // per pattern: the column-mask sequence the automaton walks
  std::vector<std::vector<uint64_t>> seq(rs->patterns.size());
  std::vector<std::vector<uint32_t>> starts(kFastCols);  // patterns whose first mask holds column v
  for (size_t pi = 0; pi < rs->patterns.size(); ++pi) {
    const PatternHost& p = rs->patterns[pi];
    if (p.special) continue;
    const size_t tl = std::min<size_t>(p.lower.size(), (size_t)depth);
    for (size_t k = 0; k < tl; ++k) {
      const int b = (unsigned char)p.lower[k];
      seq[pi].push_back(1ull << ((b & 0x1F) | ((b >> 1) & 0x20)));
    }
    if (plan[pi] && p.lower.size() < (size_t)depth) {
      const size_t e = std::min<size_t>({p.ext_cols.size(), (size_t)plan[pi], (size_t)depth - p.lower.size()});
      for (size_t j = 0; j < e; ++j) seq[pi].push_back(p.ext_cols[j]);
      ac.fast_ext[pi] = (uint8_t)e;
    }
    for (uint32_t v = 0; v < kFastCols; ++v)
      if (!seq[pi].empty() && ((seq[pi][0] >> v) & 1)) starts[v].push_back((uint32_t)pi);
  }
  using Item = uint32_t;  // pattern << 4 | columns matched (1..7)
  struct Key {
    std::vector<Item> items;
    std::vector<uint16_t> outs;
    bool operator<(const Key& o) const { return items != o.items ? items < o.items : outs < o.outs; }
  };
  std::map<Key, int> ids;
  std::vector<Key> states;
  states.push_back(Key{});
  ids[states[0]] = 0;
  std::vector<std::vector<int>> go;
  for (size_t s = 0; s < states.size(); ++s) {
    if (states.size() > max_rows) return false;
    go.emplace_back(kFastCols, 0);
    const std::vector<Item> cur = states[s].items;
    for (uint32_t v = 0; v < kFastCols; ++v) {
      Key k;
      auto advance = [&](uint32_t pi, uint32_t i) {  // pattern pi matched i columns, column v next
        if (!((seq[pi][i] >> v) & 1)) return;
        if (i + 1 == seq[pi].size()) k.outs.push_back((uint16_t)pi);
        else k.items.push_back((pi << 4) | (i + 1));
      };
      for (Item it : cur) advance(it >> 4, it & 15);
      for (uint32_t pi : starts[v]) advance(pi, 0);
      std::sort(k.items.begin(), k.items.end());
      k.items.erase(std::unique(k.items.begin(), k.items.end()), k.items.end());
      std::sort(k.outs.begin(), k.outs.end());
      k.outs.erase(std::unique(k.outs.begin(), k.outs.end()), k.outs.end());
      auto it = ids.find(k);
      int t;
      if (it != ids.end()) {
        t = it->second;
      } else {
        t = (int)states.size();
        ids.emplace(k, t);
        states.push_back(std::move(k));
      }
      go[s][v] = t;
    }
  }
  const int S = (int)states.size();
  if ((size_t)S > max_rows) return false;
  // keyword states: output states whose every output (at most kFastKwPer) is
  // a keyword-only pattern -- a keyword some non-implied gate needs, no anchor
  // role, not truncated, no class extension, printable ASCII -- so the scan
  // confirms it on the real bytes and ORs the file's keyword bit itself (no
  // k_report event: the 2-3 letter keywords jwt / lob / key of the builtin
  // rules were most of configs[2]'s 6.3 M events).  At most kFastKwBits
  // keywords and kFastKwStates states; the rest stay events.
  auto kw_simple = [&](uint32_t pi) {
    const PatternHost& p = rs->patterns[pi];
    if (p.special || p.kw < 0 || !p.kw_needed || !p.rules.empty() || p.lower.size() > (size_t)depth ||
        p.lower.size() > 8 || seq[pi].size() != p.lower.size())
      return false;
    for (unsigned char c : p.lower)
      if (c < 0x20 || c >= 0x7F) return false;
    return true;
  };
  std::vector<int> kw_bit_of(rs->keywords.size(), -1);
  std::vector<uint16_t> kw_map;
  std::vector<char> is_kw(S, 0);
  int n_kw = 0;
  // shortest keywords first (the most frequent in text: 'sk', then jwt /
  // key / lob ...): they get the low numbers, which a lane's seen-prefix test
  // (kw_resolve) needs to skip repeats
  std::vector<std::pair<size_t, int>> cand;
  for (int st = 0; st < S; ++st) {
    const auto& o = states[st].outs;
    if (o.empty() || o.size() > kFastKwPer) continue;
    bool ok = true;
    size_t len = 8;
    for (auto pi : o) {
      ok &= kw_simple(pi);
      len = std::min(len, rs->patterns[pi].lower.size());
    }
    if (ok) cand.emplace_back(len, st);
  }
  std::stable_sort(cand.begin(), cand.end());
  std::vector<int> kw_order;
  for (auto& [len, st] : cand) {
    (void)len;
    const auto& o = states[st].outs;
    if (n_kw >= (int)kFastKwStates) break;
    int need = 0;
    for (auto pi : o) need += kw_bit_of[rs->patterns[pi].kw] < 0;
    if ((int)kw_map.size() + need > (int)kFastKwBits) continue;
    for (auto pi : o)
      if (kw_bit_of[rs->patterns[pi].kw] < 0) {
        kw_bit_of[rs->patterns[pi].kw] = (int)kw_map.size();
        kw_map.push_back((uint16_t)rs->patterns[pi].kw);
      }
    is_kw[st] = 1;
    kw_order.push_back(st);
    ++n_kw;
  }
  // renumber: start first, states without outputs, keyword states, then the
  // other output states (events)
  std::vector<int> perm(S), inv;
  for (int st = 0; st < S; ++st)
    if (states[st].outs.empty()) { perm[st] = (int)inv.size(); inv.push_back(st); }
  const int first_out = (int)inv.size();
  for (int st : kw_order) { perm[st] = (int)inv.size(); inv.push_back(st); }
  const int first_ev = (int)inv.size();
  for (int st = 0; st < S; ++st)
    if (!states[st].outs.empty() && !is_kw[st]) { perm[st] = (int)inv.size(); inv.push_back(st); }
  const size_t img = ((size_t)S * kFastRowBytes + 3) & ~(size_t)3;
  ac.fast.assign(img, 0);
  ac.fast_out_off.assign(S + 1, 0);
  for (int n = 0; n < S; ++n) {
    uint16_t* row = reinterpret_cast<uint16_t*>(ac.fast.data() + (size_t)n * kFastRowBytes);
    for (uint32_t v = 0; v < kFastCols; ++v) row[v] = (uint16_t)perm[go[inv[n]][v]];
    ac.fast_out_off[n] = (uint32_t)ac.fast_out_pat.size();
    for (auto x : states[inv[n]].outs) ac.fast_out_pat.push_back(x);
  }
  ac.fast_out_off[S] = (uint32_t)ac.fast_out_pat.size();
  ac.fast_out_entry = (uint32_t)first_out;
  ac.fast_ev_entry = (uint32_t)first_ev;
  ac.fast_states = (uint32_t)S;
  {  // the keyword states' records (pattern window as PatDev::lo64 / m64: ext 0, len <= depth)
    std::vector<FastKwRec> recs((size_t)(first_ev - first_out) * kFastKwPer, FastKwRec{1, 0, 0, 0});
    for (int n = first_out; n < first_ev; ++n) {
      const auto& o = states[inv[n]].outs;
      for (size_t q = 0; q < o.size(); ++q) {
        const PatternHost& p = rs->patterns[o[q]];
        FastKwRec r{0, 0, (uint32_t)kw_bit_of[p.kw], 1};
        const size_t tl = p.lower.size();
        for (size_t k = 0; k < tl; ++k) {
          const int sh = 8 * (int)(8 - tl + k);
          r.lo64 |= (uint64_t)(uint8_t)p.lower[k] << sh;
          r.m64 |= 0xFFull << sh;
        }
        recs[(size_t)(n - first_out) * kFastKwPer + q] = r;
      }
    }
    ac.fast_kw.assign((const uint8_t*)recs.data(), (const uint8_t*)(recs.data() + recs.size()));
    ac.fast_kw_map = kw_map;
  }
  ac.fast_pair.clear();
  bool one_step_out = false;  // (a pair step skips the middle state: it must never be an output)
  for (uint32_t v = 0; v < kFastCols; ++v) one_step_out |= perm[go[0][v]] >= first_out;
  if (!one_step_out) {
    ac.fast_pair.assign(kFastCols * kFastCols, 0);
    for (uint32_t v1 = 0; v1 < kFastCols; ++v1)
      for (uint32_t v2 = 0; v2 < kFastCols; ++v2) ac.fast_pair[v1 * kFastCols + v2] = (uint16_t)perm[go[go[0][v1]][v2]];
  }
  return true;
}

// The deepest trie (<= kAcMaxLit) whose automaton fits k_scan_fast's LDS
// image; longer patterns are confirmed on hit.  Falls back to depth
// kAcMaxLit for the generic kernel when none fits.
//
// Scan-automaton extensions are tried longest first at each depth: they cut
// the scan's events (and k_report's work) by the selectivity of the classes.
bool build_ac(tsg_ruleset* rs, std::string* err) {
  for (int d = kAcMaxLit; d >= 4; --d) {
    if (!build_ac_depth(rs, d, err)) return false;
    std::vector<uint8_t> plan(rs->patterns.size(), 0);
    if (!build_fast(rs, d, plan)) continue;
    // greedy, shortest literals first (the frequent ones): extend every
    // literal shorter than t to t columns where the automaton still fits
    for (int t = 3; t <= kFastExtTo; ++t) {
      std::vector<uint8_t> want = plan;
      std::vector<size_t> grow;
      for (size_t pi = 0; pi < rs->patterns.size(); ++pi) {
        const PatternHost& p = rs->patterns[pi];
        const size_t e = std::min<size_t>(p.ext_cols.size(), p.lower.size() < (size_t)t ? t - p.lower.size() : 0);
        if (e > want[pi]) {
          want[pi] = (uint8_t)e;
          grow.push_back(pi);
        }
      }
      if (grow.empty()) continue;
      if (build_fast(rs, d, want)) {
        plan = want;
        continue;
      }
      std::stable_sort(grow.begin(), grow.end(), [&](size_t a, size_t b) {
        return rs->patterns[a].lower.size() < rs->patterns[b].lower.size();
      });
      for (size_t pi : grow) {
        std::vector<uint8_t> one = plan;
        one[pi] = want[pi];
        if (build_fast(rs, d, one)) plan = one;
      }
      break;
    }
    if (!build_fast(rs, d, plan)) return false;  // cannot happen: plan was built
    return true;
  }
  return build_ac_depth(rs, kAcMaxLit, err);
}
}  // namespace tsg

using namespace tsg;

static int add_regex(tsg_ruleset* rs, const char* src, std::string* err) {
  // one program per distinct source (custom rule sets repeat path and allow regexes)
  auto it = rs->regex_ids.find(src);
  if (it != rs->regex_ids.end()) return it->second;
  RegexHost r;
  r.src = src;
  if (!gre::compile(r.src, &r.c, err)) {
    *err = "regexp compile error: " + *err;
    return -1;
  }
  rs->regexes.push_back(std::move(r));
  rs->regex_ids[src] = (int)rs->regexes.size() - 1;
  return (int)rs->regexes.size() - 1;
}

static int add_pattern(tsg_ruleset* rs, const std::string& lower) {
  for (size_t i = 0; i < rs->patterns.size(); ++i)
    if (rs->patterns[i].lower == lower) return (int)i;
  PatternHost p;
  p.lower = lower;
  p.req.assign(lower.size(), '\0');
  rs->patterns.push_back(p);
  return (int)rs->patterns.size() - 1;
}

extern "C" {

const char* tsg_last_error(void) { return g_last_error.c_str(); }

int tsg_ruleset_compile(const tsg_rule* rules, size_t n_rules, const tsg_allow_rule* allow_rules,
                        size_t n_allow_rules, const char* const* exclude_regexes,
                        size_t n_exclude_regexes, tsg_ruleset** out, char* err, size_t errlen) {
  if (!out || (n_rules && !rules)) {
    set_err(err, errlen, "invalid argument");
    return TSG_ERR_INVALID_ARG;
  }
  *out = nullptr;
  auto* rs = new tsg_ruleset();
  rs->id = g_ruleset_ids.fetch_add(1);
  std::string e;
  auto fail = [&](int code) {
    set_err(err, errlen, e);
    delete rs;
    return code;
  };
  for (size_t i = 0; i < n_allow_rules; ++i) {
    if (allow_rules[i].regex) {
      int r = add_regex(rs, allow_rules[i].regex, &e);
      if (r < 0) return fail(TSG_ERR_REGEX);
      rs->global_allow_regex.push_back(r);
    }
    if (allow_rules[i].path) {
      int r = add_regex(rs, allow_rules[i].path, &e);
      if (r < 0) return fail(TSG_ERR_REGEX);
      rs->global_allow_path.push_back(r);
    }
  }
  for (size_t i = 0; i < n_exclude_regexes; ++i) {
    int r = add_regex(rs, exclude_regexes[i], &e);
    if (r < 0) return fail(TSG_ERR_REGEX);
    rs->global_exclude.push_back(r);
    rs->any_exclude = true;
  }
  std::map<std::string, int> kwid;
  for (size_t i = 0; i < n_rules; ++i) {
    const tsg_rule& in = rules[i];
    RuleHost r;
    r.id = in.id ? in.id : "";
    r.group_name = in.secret_group_name ? in.secret_group_name : "";
    if (in.regex) {
      r.regex = add_regex(rs, in.regex, &e);
      if (r.regex < 0) return fail(TSG_ERR_REGEX);
    }
    for (size_t k = 0; k < in.n_keywords; ++k) {
      std::string kw = in.keywords[k] ? in.keywords[k] : "", lw;
      // a keyword whose lowercase holds a non-ASCII rune is found by
      // k_uni_keywords around the batch's non-ASCII bytes, not by the automaton
      if (!go_lower_utf8(kw, &lw) || lw.find('\0') != std::string::npos) {
        e = "rule " + r.id + ": a keyword with invalid UTF-8 or NUL is outside this engine's coverage";
        return fail(TSG_ERR_UNSUPPORTED);
      }
      r.keywords.push_back(lw);
    }
    if (in.path) {
      r.path = add_regex(rs, in.path, &e);
      if (r.path < 0) return fail(TSG_ERR_REGEX);
      rs->any_path_rules = true;
    }
    for (size_t k = 0; k < in.n_allow_rules; ++k) {
      if (in.allow_rules[k].regex) {
        int x = add_regex(rs, in.allow_rules[k].regex, &e);
        if (x < 0) return fail(TSG_ERR_REGEX);
        r.allow_regex.push_back(x);
      }
      if (in.allow_rules[k].path) {
        int x = add_regex(rs, in.allow_rules[k].path, &e);
        if (x < 0) return fail(TSG_ERR_REGEX);
        r.allow_path.push_back(x);
        rs->any_path_rules = true;
      }
    }
    for (size_t k = 0; k < in.n_exclude_regexes; ++k) {
      int x = add_regex(rs, in.exclude_regexes[k], &e);
      if (x < 0) return fail(TSG_ERR_REGEX);
      r.exclude.push_back(x);
      rs->any_exclude = true;
    }
    if (r.regex < 0) {
      r.mode = MODE_NEVER;
    } else {
      const gre::Compiled& c = rs->regexes[r.regex].c;
      bool has_group = true;
      if (!r.group_name.empty()) {
        has_group = false;
        for (auto& nm : c.prog.cap_names) has_group |= (nm == r.group_name);
      }
      if (has_group && !r.group_name.empty() && (uint32_t)c.prog.ncap > kMaxCap) {
        e = "rule " + r.id + ": too many capture groups for the secret-group extractor";
        return fail(TSG_ERR_UNSUPPORTED);
      }
      // secret group from the match span alone (k_verify emit_match): one
      // group of that name whose position gre::group_span pins
      if (has_group && !r.group_name.empty()) {
        int slot = -1, count = 0;
        for (size_t k = 0; k < c.prog.cap_names.size(); ++k)
          if (c.prog.cap_names[k] == r.group_name) slot = (int)k, ++count;
        if (count == 1) r.grp = gre::group_span(c.prog, (uint32_t)slot);
        if (count == 1 && !r.grp.valid) r.grun = gre::group_run(c.prog, (uint32_t)slot, r.grp.len);
      }
      // no group of that name => getMatchSubgroupsLocations yields nothing
      if (!has_group) r.mode = MODE_NEVER;
      else r.mode = c.anchor.valid ? MODE_ANCHORED : MODE_FULL;
      if (r.mode == MODE_ANCHORED) {
        build_follow(c, &r.follow);
        // the verify DFA; past its state budget (or with \b, (?m) ^ $) the
        // bit-parallel Glushkov NFA (nfa.cpp), and the Pike VM only when
        // neither exists
        if (!build_dfa(c, &r.dfa)) build_nfa(c, &r.nfa);
      }
      // implied gate: every anchor literal contains one of the rule's keywords
      // (so a hit proves MatchKeywords, scanner.go:169-181)
      bool kw_ok = !r.keywords.empty();
      for (auto& kw : r.keywords) kw_ok &= !kw.empty();
      if (r.mode == MODE_ANCHORED && kw_ok) {
        bool all = !c.anchor.lits.empty();
        for (auto& l : c.anchor.lits) {
          bool has = false;
          for (auto& kw : r.keywords) has |= l.lower.find(kw) != std::string::npos;
          all &= has;
        }
        r.gate_implied = all;
      }
      if (r.mode == MODE_ANCHORED)
        for (auto& l : c.anchor.lits)
          for (size_t j = 0; j < l.lower.size(); ++j)
            r.fold_gate |= (l.lower[j] == 'k' || l.lower[j] == 's') && l.req[j] == 0;
    }
    for (auto& kw : r.keywords) {
      if (!kwid.count(kw) && !kw.empty()) {
        int id = (int)rs->keywords.size();
        kwid[kw] = id;
        rs->keywords.push_back(kw);
        rs->kw_uni.push_back(is_ascii(kw) ? 0 : 1);
      }
    }
    rs->rules.push_back(std::move(r));
  }
  // patterns: keywords, anchor literals, fold-special sequences
  for (size_t k = 0; k < rs->keywords.size(); ++k) {
    if (rs->kw_uni[k]) continue;
    int p = add_pattern(rs, rs->keywords[k]);
    rs->patterns[p].kw = (int)k;
  }
  static const char* kSpecial[] = {"\xC4\xB0", "\xC5\xBF", "\xE2\x84\xAA"};
  for (auto* s : kSpecial) {
    int p = add_pattern(rs, s);
    rs->patterns[p].special = true;
  }
  for (size_t ri = 0; ri < rs->rules.size(); ++ri) {
    RuleHost& r = rs->rules[ri];
    if (r.mode != MODE_ANCHORED) continue;
    const gre::Anchor& a = rs->regexes[r.regex].c.anchor;
    for (auto& lit : a.lits) {
      int p = add_pattern(rs, lit.lower);
      PatternHost& ph = rs->patterns[p];
      bool has_req = false;
      for (char c : lit.req) has_req |= c != '\0';
      if (!ph.any_anchor) {
        ph.req = lit.req;
        ph.confirm = has_req;
      } else if (ph.confirm && (!has_req || ph.req != lit.req)) {
        ph.confirm = false;  // differing case requirements: record every hit
      }
      ph.any_anchor = true;
      if (std::find(ph.rules.begin(), ph.rules.end(), (uint32_t)ri) == ph.rules.end())
        ph.rules.push_back((uint32_t)ri);
    }
  }
  if (rs->patterns.size() >= 4095) {  // build_fast items: pattern << 4
    e = "too many keyword/anchor literals";
    return fail(TSG_ERR_UNSUPPORTED);
  }
  // scan-automaton extensions: for anchor-only patterns (no keyword some
  // non-implied gate needs), the column sets every anchored use requires next
  {
    std::vector<uint8_t> kw_needed(rs->keywords.size(), 0);
    for (auto& r : rs->rules)
      if (!r.gate_implied || r.fold_gate)  // the same set engine.hip marks kw_needed
        for (auto& kw : r.keywords)
          for (size_t k = 0; k < rs->keywords.size(); ++k)
            if (!kw.empty() && rs->keywords[k] == kw) kw_needed[k] = 1;
    for (auto& ph : rs->patterns) {
      ph.kw_needed = ph.kw >= 0 && kw_needed[ph.kw];
      if (ph.special || ph.rules.empty() || (ph.kw >= 0 && kw_needed[ph.kw])) continue;
      bool first = true;
      for (uint32_t ri : ph.rules) {
        const gre::Compiled& c = rs->regexes[rs->rules[ri].regex].c;
        for (auto& lit : c.anchor.lits) {
          if (lit.lower != ph.lower) continue;
          std::vector<uint64_t> cols = follow_ext(c, lit, kAcMaxLit);
          if (first) {
            ph.ext_cols = cols;
            first = false;
          } else {
            if (cols.size() < ph.ext_cols.size()) ph.ext_cols.resize(cols.size());
            for (size_t j = 0; j < ph.ext_cols.size(); ++j) ph.ext_cols[j] |= cols[j];
          }
        }
      }
    }
  }
  if (!build_ac(rs, &e)) return fail(TSG_ERR_UNSUPPORTED);
  if (int rc = big_blob_precheck(rs->ac, &e)) return fail(rc);  // (a malformed k_scan_big blob is an error, not a hang)
  {  // path regexes: MatchString as one anchored DFA walk over the path
    rs->path_dfa.assign(rs->regexes.size(), DfaHost{});
    std::vector<int> pr(rs->global_allow_path.begin(), rs->global_allow_path.end());
    for (auto& r : rs->rules) {
      if (r.path >= 0) pr.push_back(r.path);
      pr.insert(pr.end(), r.allow_path.begin(), r.allow_path.end());
    }
    // (only path regexes: AllowLocation's allow regexes run in k_allow /
    // emit_match as literal prefilter + Pike VM, which need no DFA)
    for (int x : pr) {
      if (rs->path_dfa[x].valid) continue;
      gre::Compiled any;
      std::string err2;
      if (gre::compile("(?s:.)*?(?:" + rs->regexes[x].src + ")", &any, &err2)) build_dfa(any, &rs->path_dfa[x]);
    }
    // the global allow paths as one alternation (each regex's flags stay
    // inside its own group), for Required's per-file AllowPath on the host
    if (rs->global_allow_path.size() > 1) {
      std::string u = "(?s:.)*?(?:";
      for (size_t k = 0; k < rs->global_allow_path.size(); ++k)
        u += (k ? "|(?:" : "(?:") + rs->regexes[rs->global_allow_path[k]].src + ")";
      u += ")";
      gre::Compiled any;
      std::string err2;
      if (gre::compile(u, &any, &err2)) build_dfa(any, &rs->allow_path_union);
    }
  }
  *out = rs;
  return TSG_OK;
}

void tsg_ruleset_free(tsg_ruleset* rs) { delete rs; }

tsg_ruleset::~tsg_ruleset() { delete gate_rs; }



size_t tsg_ruleset_rule_count(const tsg_ruleset* rs) { return rs ? rs->rules.size() : 0; }

int tsg_ruleset_rule_info(const tsg_ruleset* rs, size_t i, int* mode, uint32_t* amin,
                          uint32_t* amax, size_t* nlits) {
  if (!rs || i >= rs->rules.size()) return TSG_ERR_INVALID_ARG;
  const RuleHost& r = rs->rules[i];
  if (mode) *mode = r.mode;
  const gre::Anchor* a = r.regex >= 0 ? &rs->regexes[r.regex].c.anchor : nullptr;
  if (amin) *amin = a && a->valid ? a->off_min : 0;
  if (amax) *amax = a && a->valid ? a->off_max : 0;
  if (nlits) *nlits = a && a->valid ? a->lits.size() : 0;
  return TSG_OK;
}

// Anchor literal k of rule i: lowercased bytes and the case requirement
// (0 = either case), both `len` bytes long (diagnostics / candidate studies).
int tsg_ruleset_rule_literal(const tsg_ruleset* rs, size_t i, size_t k, char* lower, char* req, size_t cap,
                             size_t* len) {
  if (!rs || i >= rs->rules.size() || !len) return TSG_ERR_INVALID_ARG;
  const RuleHost& r = rs->rules[i];
  const gre::Anchor* a = r.regex >= 0 ? &rs->regexes[r.regex].c.anchor : nullptr;
  if (!a || !a->valid || k >= a->lits.size()) return TSG_ERR_INVALID_ARG;
  const gre::Lit& L = a->lits[k];
  *len = L.lower.size();
  if (cap < L.lower.size()) return TSG_ERR_INVALID_ARG;
  if (lower) memcpy(lower, L.lower.data(), L.lower.size());
  if (req) memcpy(req, L.req.data(), L.req.size());
  return TSG_OK;
}

// Scan-automaton pattern k (diagnostics / soundness tests): its lowercased
// literal, the class positions k_scan_fast's automaton requires after it
// (*ext, 0 without a fast image) and their fold-column masks (cols[0..ext)).
int tsg_ruleset_scan_pattern(const tsg_ruleset* rs, size_t k, char* lower, size_t cap, size_t* len, uint32_t* ext,
                             uint64_t* cols, uint32_t* fast_states) {
  if (!rs || k >= rs->patterns.size() || !len) return TSG_ERR_INVALID_ARG;
  const PatternHost& p = rs->patterns[k];
  *len = p.lower.size();
  if (lower) {
    if (cap < p.lower.size()) return TSG_ERR_INVALID_ARG;
    memcpy(lower, p.lower.data(), p.lower.size());
  }
  const uint32_t e = rs->ac.fast.empty() ? 0 : rs->ac.fast_ext[k];
  if (ext) *ext = e;
  if (cols)
    for (uint32_t j = 0; j < e; ++j) cols[j] = p.ext_cols[j];
  if (fast_states) *fast_states = rs->ac.fast_states;
  return TSG_OK;
}

// k_scan_fast's LDS image (diagnostics / layout studies): copies up to cap
// bytes, *len = image bytes (0 = no fast image), *out_entry = first output
// state's entry (entries are row offsets / 2).
int tsg_ruleset_scan_image(const tsg_ruleset* rs, uint8_t* buf, size_t cap, size_t* len, uint32_t* out_entry) {
  if (!rs || !len) return TSG_ERR_INVALID_ARG;
  *len = rs->ac.fast.size();
  if (out_entry) *out_entry = rs->ac.fast_out_entry;
  if (buf) memcpy(buf, rs->ac.fast.data(), std::min(cap, rs->ac.fast.size()));
  return TSG_OK;
}

// k_scan_fast's keyword states (diagnostics): their count and the keywords
// (lowercased, NUL-separated into buf) whose bits the scan sets itself.
int tsg_ruleset_kw_states(const tsg_ruleset* rs, uint32_t* n_states, uint32_t* n_keywords, char* buf, size_t cap) {
  if (!rs || !n_states || !n_keywords) return TSG_ERR_INVALID_ARG;
  *n_states = rs->ac.fast.empty() ? 0 : rs->ac.fast_ev_entry - rs->ac.fast_out_entry;
  *n_keywords = (uint32_t)rs->ac.fast_kw_map.size();
  size_t at = 0;
  for (uint16_t k : rs->ac.fast_kw_map) {
    const std::string& w = rs->keywords[k];
    if (buf && at + w.size() + 1 <= cap) {
      memcpy(buf + at, w.data(), w.size());
      buf[at + w.size()] = 0;
    }
    at += w.size() + 1;
  }
  return TSG_OK;
}

// Program size of rule i's regex (diagnostics: VM scratch sizing).
int tsg_ruleset_rule_prog(const tsg_ruleset* rs, size_t i, uint32_t* n_inst, uint32_t* n_cap) {
  if (!rs || i >= rs->rules.size()) return TSG_ERR_INVALID_ARG;
  const RuleHost& r = rs->rules[i];
  if (n_inst) *n_inst = r.regex >= 0 ? (uint32_t)rs->regexes[r.regex].c.prog.inst.size() : 0;
  if (n_cap) *n_cap = r.regex >= 0 ? (uint32_t)rs->regexes[r.regex].c.prog.ncap : 0;
  return TSG_OK;
}

// Secret-group span rule of rule i (gre::group_span; what k_verify uses to
// skip the capture search): *valid = 0 when the capture search decides.
int tsg_ruleset_group_span(const tsg_ruleset* rs, size_t i, int* valid, int* pre, int* len, int* suf) {
  if (!rs || i >= rs->rules.size() || !valid) return TSG_ERR_INVALID_ARG;
  const gre::GroupSpan& g = rs->rules[i].grp;  // exactly what upload_ruleset hands the device
  *valid = g.valid ? 1 : 0;
  if (pre) *pre = g.pre;
  if (len) *len = g.len;
  if (suf) *suf = g.suf;
  return TSG_OK;
}

// Byte-run group rule of rule i (gre::group_run, used when group_span is not
// valid): *valid = 0 when neither shortcut applies; masks = 4 u32 words each.
int tsg_ruleset_group_run(const tsg_ruleset* rs, size_t i, int* valid, int* len, uint32_t* s_alpha,
                          uint32_t* b_alpha) {
  if (!rs || i >= rs->rules.size() || !valid) return TSG_ERR_INVALID_ARG;
  const gre::GroupRun& g = rs->rules[i].grun;  // exactly what upload_ruleset hands the device
  *valid = g.valid ? 1 : 0;
  if (len) *len = g.len;
  for (int k = 0; k < 4; ++k) {
    if (s_alpha) s_alpha[k] = g.s_alpha[k];
    if (b_alpha) b_alpha[k] = g.b_alpha[k];
  }
  return TSG_OK;
}

// Verify DFA of rule i on host text: 1 = match [s, *me), 0 = none, 2 = not
// decidable by the DFA (no DFA, byte >= 0x80, s at the end) -> Pike VM.
int tsg_ruleset_dfa_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t s,
                          int* result, size_t* me, uint32_t* n_states) {
  if (!rs || i >= rs->rules.size() || !result) return TSG_ERR_INVALID_ARG;
  const DfaHost& d = rs->rules[i].dfa;
  if (n_states) *n_states = d.valid ? d.nstates : 0;
  size_t e = 0;
  *result = dfa_anchored(d, text, len, s, &e);
  if (me) *me = e;
  return TSG_OK;
}

// MatchString of rule i's path regex (which = 0), its first allow-path regex
// (which = 1) or the i-th global allow path (which = 2) through the path DFA
// k_path_gate walks (ruleset path_dfa):
// *result 1 = match, 0 = none, 2 = no DFA / undecidable (the Pike VM decides).
int tsg_ruleset_path_dfa_check(const tsg_ruleset* rs, size_t i, int which, const uint8_t* path, size_t len,
                               int* result) {
  if (!rs || !result || (len && !path)) return TSG_ERR_INVALID_ARG;
  int x = -1;
  if (which == 2) {  // i-th global allow path
    if (i >= rs->global_allow_path.size()) return TSG_ERR_INVALID_ARG;
    x = rs->global_allow_path[i];
  } else {
    if (i >= rs->rules.size()) return TSG_ERR_INVALID_ARG;
    const RuleHost& r = rs->rules[i];
    x = which == 0 ? r.path : (r.allow_path.empty() ? -1 : r.allow_path[0]);
  }
  *result = 2;
  if (x < 0 || (size_t)x >= rs->path_dfa.size() || !rs->path_dfa[x].valid) return TSG_OK;
  size_t e = 0;
  *result = dfa_anchored(rs->path_dfa[x], path, len, 0, &e);
  return TSG_OK;
}

// Bit-parallel NFA of rule i on host text (nfa_walk_host): threads started
// at every boundary in [s, inj_hi]; *result 1 = match (anchored: the only end
// *me; unanchored: the first end), 0 = none, 2 = the Pike VM decides;
// *n_pos = its positions (0 = the rule has no NFA).
int tsg_ruleset_nfa_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t s, size_t inj_hi,
                          int* result, size_t* me, uint32_t* n_pos) {
  if (!rs || i >= rs->rules.size() || !result || inj_hi < s) return TSG_ERR_INVALID_ARG;
  const NfaHost& d = rs->rules[i].nfa;
  if (n_pos) *n_pos = d.valid ? d.npos : 0;
  size_t e = 0;
  *result = nfa_walk_host(d, text, len, s, inj_hi, &e);
  if (me) *me = e;
  return TSG_OK;
}

// Candidate filter of rule i on host text (diagnostics / soundness tests):
// *accept = 0 only if no match of the rule can contain an anchor hit at h.
// *n_states = the filter's DFA states (0 = rule has no filter).
int tsg_ruleset_follow_check(const tsg_ruleset* rs, size_t i, const uint8_t* text, size_t len, size_t h,
                             int* accept, uint32_t* n_states) {
  if (!rs || i >= rs->rules.size()) return TSG_ERR_INVALID_ARG;
  const FollowDfa& f = rs->rules[i].follow;
  if (n_states) *n_states = f.valid ? f.nstates : 0;
  if (accept) *accept = follow_accepts(f, text, len, h) ? 1 : 0;
  return TSG_OK;
}

// ---- host regex diagnostics (compiler + VM on the CPU) ---------------------
struct HostVm {
  std::vector<uint16_t> sp0, sp1, d0, d1, stk;
  std::vector<uint32_t> s0, s1;
  gre::VmScratch sc;
  explicit HostVm(size_t n) : sp0(n), sp1(n), d0(n), d1(n), stk(n + 1), s0(n), s1(n) {
    sc.sparse[0] = sp0.data();
    sc.sparse[1] = sp1.data();
    sc.dense[0] = d0.data();
    sc.dense[1] = d1.data();
    sc.start[0] = s0.data();
    sc.start[1] = s1.data();
    sc.stack = stk.data();
  }
};

static gre::ProgView view_of(const gre::Prog& p) {
  return gre::ProgView{p.inst.data(), p.classes.data(), p.ranges.data(), (uint32_t)p.inst.size(),
                       p.start, (uint32_t)p.ncap, p.nvis};
}

extern "C++" namespace tsg {
// Global AllowRules.AllowPath (scanner.go:200-207) on the host: MatchString of
// every compiled global allow-path regex.  Per file, not per byte.
bool host_allow_path(const tsg_ruleset* rs, const uint8_t* path, size_t len) {
  if (rs->allow_path_union.valid) {
    size_t e = 0;
    const int d = dfa_anchored(rs->allow_path_union, path, len, 0, &e);
    if (d != 2) return d == 1;
  }
  for (int r : rs->global_allow_path) {
    // the regex's MatchString DFA (k_path_gate's) decides most paths in one
    // table walk; the Pike VM only what it cannot (non-ASCII, DFA too big)
    if ((size_t)r < rs->path_dfa.size() && rs->path_dfa[r].valid) {
      size_t e = 0;
      const int d = dfa_anchored(rs->path_dfa[r], path, len, 0, &e);
      if (d == 1) return true;
      if (d == 0) continue;
    }
    const gre::Prog& p = rs->regexes[r].c.prog;
    // per-thread VM scratch, freed when the thread exits (tsg_analyze_layer's
    // Required workers are short-lived threads)
    thread_local std::unique_ptr<HostVm> vm;
    thread_local size_t vm_n = 0;
    if (!vm || vm_n < p.inst.size()) {
      vm_n = p.inst.size() + 64;
      vm.reset(new HostVm(vm_n));
    }
    uint32_t ms, me;
    if (gre::vm_search(view_of(p), path, (uint32_t)len, 0, (uint32_t)len, true, vm->sc, &ms, &me)) return true;
  }
  return false;
}
}  // namespace tsg

int tsg_ruleset_allow_path(const tsg_ruleset* rs, const char* path, size_t len, int* allowed) {
  if (!rs || (!path && len) || !allowed) return TSG_ERR_INVALID_ARG;
  *allowed = tsg::host_allow_path(rs, (const uint8_t*)path, len) ? 1 : 0;
  return TSG_OK;
}

int tsg_regex_match(const char* pattern, const uint8_t* text, size_t len, int* matched) {
  if (!pattern || !matched) return TSG_ERR_INVALID_ARG;
  gre::Compiled c;
  std::string e;
  if (!gre::compile(pattern, &c, &e)) {
    g_last_error = e;
    return TSG_ERR_REGEX;
  }
  HostVm vm(c.prog.inst.size());
  uint32_t ms, me;
  *matched = gre::vm_search(view_of(c.prog), text, (uint32_t)len, 0, (uint32_t)len, true, vm.sc, &ms,
                            &me);
  return TSG_OK;
}

int tsg_regex_find_all(const char* pattern, const uint8_t* text, size_t len, int64_t* pairs,
                       size_t cap, size_t* n_out) {
  if (!pattern || !n_out) return TSG_ERR_INVALID_ARG;
  gre::Compiled c;
  std::string e;
  if (!gre::compile(pattern, &c, &e)) {
    g_last_error = e;
    return TSG_ERR_REGEX;
  }
  HostVm vm(c.prog.inst.size());
  gre::ProgView pv = view_of(c.prog);
  size_t n = 0;
  int64_t prev_end = -1;
  uint32_t pos = 0;
  uint32_t L = (uint32_t)len;
  // Go regexp.go allMatches
  while (pos <= L) {
    uint32_t ms, me;
    if (!gre::vm_search(pv, text, L, pos, L, false, vm.sc, &ms, &me)) break;
    bool accept = true;
    if (me == pos) {
      if ((int64_t)ms == prev_end) accept = false;
      uint32_t w;
      gre::decode_rune(text, L, pos, &w);
      pos = w > 0 ? pos + w : L + 1;
    } else {
      pos = me;
    }
    prev_end = me;
    if (accept) {
      if (n < cap) {
        pairs[2 * n] = ms;
        pairs[2 * n + 1] = me;
      }
      ++n;
    }
  }
  *n_out = n;
  return TSG_OK;
}

}  // extern "C"

namespace tsg {
const tsg_ruleset* gate_ruleset(const tsg_ruleset* rs, std::string* err) {
  std::lock_guard<std::mutex> lk(rs->gate_mu);
  if (rs->gate_rs) return rs->gate_rs;
  // rules keep their keywords (already lowercased: ToLower is idempotent on
  // them) and lose the regex; allow rules, paths and excludes do not touch
  // MatchKeywords (scanner.go:169-181)
  std::vector<tsg_rule> rules(rs->rules.size());
  std::vector<std::vector<const char*>> kws(rs->rules.size());
  for (size_t i = 0; i < rs->rules.size(); ++i) {
    const RuleHost& r = rs->rules[i];
    for (auto& k : r.keywords) kws[i].push_back(k.c_str());
    tsg_rule& t = rules[i];
    memset(&t, 0, sizeof(t));
    t.id = r.id.c_str();
    t.keywords = kws[i].data();
    t.n_keywords = kws[i].size();
  }
  tsg_ruleset* g = nullptr;
  char ebuf[512] = {0};
  if (tsg_ruleset_compile(rules.data(), rules.size(), nullptr, 0, nullptr, 0, &g, ebuf, sizeof(ebuf)) != TSG_OK) {
    *err = std::string("gate ruleset: ") + ebuf;
    return nullptr;
  }
  rs->gate_rs = g;
  return g;
}
}  // namespace tsg

extern "C" int tsg_ruleset_stats(const tsg_ruleset* rs, uint32_t* n_states, uint32_t* n_classes,
                                 uint32_t* n_patterns, uint32_t* n_keywords, int* fast_path) {
  if (!rs) return TSG_ERR_INVALID_ARG;
  if (n_states) *n_states = rs->ac.nstates;
  if (n_classes) *n_classes = rs->ac.nclasses;
  if (n_patterns) *n_patterns = (uint32_t)rs->patterns.size();
  if (n_keywords) *n_keywords = (uint32_t)rs->keywords.size();
  if (fast_path) *fast_path = rs->ac.fast.empty() ? 0 : 1;
  return TSG_OK;
}
