// nfa.cpp — per-rule bit-parallel Glushkov NFA for k_verify (BASELINE.json
// north_star (1): "a bit-parallel Glushkov/shift-and NFA fallback when a
// rule's DFA state count explodes").
//
// The verify DFA (dfa.cpp) is a subset construction over ordered thread
// lists; patterns like `(?:x|y)*x(?:x|y){k}lit` (a gitleaks-style rule family
// of configs[4]) need 2^k states for it, and it does not model \b / \B or
// (?m) ^ $.  Those rules used to run Go's Pike VM per candidate window
// (pikevm.h) -- one global-memory thread queue per lane, ~10^3 dependent L2
// accesses per byte.  Here the same program runs as a Glushkov automaton in
// two 64-bit words per lane:
//
//   positions  the consuming instructions (I_RUNE, I_RUNE1, I_ANY, I_ANYNL)
//              reachable from the start, numbered in program order, <= 128;
//   first      positions an epsilon path from the start reaches;
//   follow(p)  positions an epsilon path from p.out reaches;
//   last       positions whose out reaches MATCH;
//   an epsilon path through I_EMPTY carries the EmptyOp flags it needs at the
//   boundary it is taken (Go's machine.add context): such edges are kept
//   apart as conditional masks and checked against empty_ctx there.
//
// The follow relation is stored LimEx-style (Hyperscan's "limited exception"
// NFAs): the kNfaShifts most common deltas q - p become (mask, shift) pairs,
// every other edge lives in a per-position exception record.  nfa_walk.h runs
// it; leftmost-first exactness is kept by the caller (k_verify tests starts
// in increasing order and takes a start's end only when it is the ONLY end a
// match from that start can have; else the VM decides that one start).
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <vector>

#include "engine.h"
#include "nfa_walk.h"

namespace tsg {
namespace {

using gre::Inst;

bool is_consuming(const Inst& in) {
  return in.op == gre::I_RUNE || in.op == gre::I_RUNE1 || in.op == gre::I_ANY || in.op == gre::I_ANYNL;
}

bool consumes_ascii(const gre::Prog& p, const Inst& in, int c) {
  switch (in.op) {
    case gre::I_RUNE: {
      const gre::ClassDesc& cd = p.classes[in.arg];
      return (cd.ascii[c >> 5] >> (c & 31)) & 1;
    }
    case gre::I_RUNE1: return (int)in.arg == c;
    case gre::I_ANY: return true;
    case gre::I_ANYNL: return c != '\n';
  }
  return false;
}

// Non-ASCII rune symbols (dfa.cpp's): K, ſ, İ, U+FFFD, then "any other rune".
constexpr uint32_t kSymRune[kDfaRuneSyms - 1] = {0x212A, 0x17F, 0x130, 0xFFFD};

bool class_has(const gre::Prog& p, const gre::ClassDesc& cd, uint32_t r) {
  for (uint32_t k = 0; k < cd.nranges; ++k)
    if (p.ranges[cd.range_off + 2 * k] <= r && r <= p.ranges[cd.range_off + 2 * k + 1]) return true;
  return false;
}

bool consumes_rune(const gre::Prog& p, const Inst& in, uint32_t r) {
  switch (in.op) {
    case gre::I_RUNE: return class_has(p, p.classes[in.arg], r);
    case gre::I_RUNE1: return in.arg == r;
    case gre::I_ANY:
    case gre::I_ANYNL: return true;
  }
  return false;
}

// Non-ASCII runes other than kSymRune an instruction consumes: 0 none, -1 all,
// 1 some (then "other" is not one symbol for this program).
int other_runes(const gre::Prog& p, const Inst& in) {
  auto in_dom = [](uint64_t r) { return r >= 0x80 && r <= 0x10FFFF && !(r >= 0xD800 && r <= 0xDFFF); };
  const uint64_t dom = (0x10FFFF - 0x80 + 1) - 0x800 - (kDfaRuneSyms - 1);
  switch (in.op) {
    case gre::I_ANY:
    case gre::I_ANYNL: return -1;
    case gre::I_RUNE1: {
      if (!in_dom(in.arg)) return 0;
      for (uint32_t r : kSymRune)
        if (r == in.arg) return 0;
      return 1;
    }
    case gre::I_RUNE: {
      const gre::ClassDesc& cd = p.classes[in.arg];
      uint64_t cnt = 0;
      for (uint32_t k = 0; k < cd.nranges; ++k) {
        const uint64_t lo = std::max<uint64_t>(p.ranges[cd.range_off + 2 * k], 0x80);
        const uint64_t hi = std::min<uint64_t>(p.ranges[cd.range_off + 2 * k + 1], 0x10FFFF);
        if (lo > hi) continue;
        cnt += hi - lo + 1;
        const uint64_t slo = std::max<uint64_t>(lo, 0xD800), shi = std::min<uint64_t>(hi, 0xDFFF);
        if (slo <= shi) cnt -= shi - slo + 1;
        for (uint32_t r : kSymRune)
          if (r >= lo && r <= hi && in_dom(r)) --cnt;
      }
      return cnt == 0 ? 0 : cnt == dom ? -1 : 1;
    }
  }
  return 0;
}

constexpr int kMatchTarget = -2;

// Epsilon closure from pc0: every (target, required EmptyOp flags) pair, the
// target a position index or kMatchTarget.  Paths are explored with their
// accumulated flags, so a target reached both freely and through an
// assertion appears with both.
std::vector<std::pair<int, uint32_t>> closure(const gre::Prog& p, const std::vector<int>& pos_of, uint32_t pc0) {
  std::vector<std::pair<int, uint32_t>> out;
  std::set<std::pair<uint32_t, uint32_t>> seen;
  std::vector<std::pair<uint32_t, uint32_t>> stk{{pc0, 0u}};
  while (!stk.empty()) {
    auto [pc, r] = stk.back();
    stk.pop_back();
    while (pc != 0 && pc < p.inst.size() && seen.insert({pc, r}).second) {
      const Inst& in = p.inst[pc];
      if (in.op == gre::I_ALT) {
        stk.push_back({in.arg, r});
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_EMPTY) {
        r |= in.empty;
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_NOP || in.op == gre::I_CAP) {
        pc = in.out;
        continue;
      }
      if (in.op == gre::I_MATCH) out.push_back({kMatchTarget, r});
      else if (is_consuming(in)) out.push_back({pos_of[pc], r});
      break;
    }
  }
  // a target reached without a condition needs none
  std::set<int> free_t;
  for (auto& t : out)
    if (t.second == 0) free_t.insert(t.first);
  std::vector<std::pair<int, uint32_t>> res;
  std::set<std::pair<int, uint32_t>> uniq;
  for (auto& t : out)
    if ((t.second == 0 || !free_t.count(t.first)) && uniq.insert(t).second) res.push_back(t);
  return res;
}

void set_bit(U128& m, int i) {
  if (i < 64) m.lo |= 1ull << i;
  else m.hi |= 1ull << (i - 64);
}

// conditional masks grouped by required flags (at most kNfaMaxCond groups)
bool add_cond(std::vector<std::pair<uint32_t, U128>>& groups, uint32_t r, int bit) {
  for (auto& g : groups)
    if (g.first == r) {
      set_bit(g.second, bit);
      return true;
    }
  if (groups.size() >= kNfaMaxCond) return false;
  groups.push_back({r, U128{0, 0}});
  set_bit(groups.back().second, bit);
  return true;
}

}  // namespace

bool build_nfa(const gre::Compiled& c, NfaHost* out) {
  *out = NfaHost{};
  const gre::Prog& p = c.prog;
  if (p.inst.empty() || p.start == 0 || c.can_match_empty || c.min_len == 0) return false;
  // reachable consuming instructions, in program order
  std::vector<uint8_t> reach_pc(p.inst.size(), 0);
  {
    std::vector<uint32_t> stk{p.start};
    while (!stk.empty()) {
      const uint32_t pc = stk.back();
      stk.pop_back();
      if (pc == 0 || pc >= p.inst.size() || reach_pc[pc]) continue;
      reach_pc[pc] = 1;
      const Inst& in = p.inst[pc];
      if (in.op == gre::I_MATCH || in.op == gre::I_FAIL) continue;
      stk.push_back(in.out);
      if (in.op == gre::I_ALT) stk.push_back(in.arg);
    }
  }
  std::vector<int> pos_of(p.inst.size(), -1);
  std::vector<uint32_t> pcs;
  for (uint32_t pc = 0; pc < p.inst.size(); ++pc)
    if (reach_pc[pc] && is_consuming(p.inst[pc])) {
      pos_of[pc] = (int)pcs.size();
      pcs.push_back(pc);
    }
  const uint32_t m = (uint32_t)pcs.size();
  if (m == 0 || m > kNfaMaxPos) return false;

  NfaDev N{};
  N.npos = m;
  std::vector<std::pair<uint32_t, U128>> first_c, last_c;
  for (auto& t : closure(p, pos_of, p.start)) {
    if (t.first == kMatchTarget) return false;  // an empty match (conditional or not): the VM's case
    if (t.second == 0) set_bit(N.first_u, t.first);
    else if (!add_cond(first_c, t.second, t.first)) return false;
  }
  // follow edges; conditional ones become exception edges
  struct Edge {
    int from, to;
  };
  std::vector<Edge> free_edges;
  std::vector<std::vector<std::pair<uint32_t, int>>> cond_edges(m);  // per position: (flags, to)
  for (uint32_t i = 0; i < m; ++i) {
    for (auto& t : closure(p, pos_of, p.inst[pcs[i]].out)) {
      if (t.first == kMatchTarget) {
        if (t.second == 0) set_bit(N.last_u, (int)i);
        else if (!add_cond(last_c, t.second, (int)i)) return false;
      } else if (t.second == 0) {
        free_edges.push_back({(int)i, t.first});
      } else {
        cond_edges[i].push_back({t.second, t.first});
      }
    }
  }
  // the most common deltas become shifts
  std::map<int, uint32_t> cnt;
  for (auto& e : free_edges) ++cnt[e.to - e.from];
  std::vector<std::pair<uint32_t, int>> by;
  for (auto& kv : cnt) by.push_back({kv.second, kv.first});
  std::sort(by.begin(), by.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
  if (by.size() > kNfaShifts) by.resize(kNfaShifts);
  std::map<int, uint32_t> slot;
  for (auto& b : by) {
    slot[b.second] = N.nshift;
    N.shift[N.nshift++] = b.second;
  }
  std::vector<U128> exc_free(m, U128{0, 0});
  std::vector<uint8_t> is_exc(m, 0);
  for (auto& e : free_edges) {
    auto it = slot.find(e.to - e.from);
    if (it != slot.end()) {
      set_bit(N.smask[it->second], e.from);
    } else {
      set_bit(exc_free[e.from], e.to);
      is_exc[e.from] = 1;
    }
  }
  for (uint32_t i = 0; i < m; ++i)
    if (!cond_edges[i].empty()) is_exc[i] = 1;
  std::vector<NfaExc> excs;
  for (uint32_t i = 0; i < kNfaMaxPos; ++i) N.exc_of[i] = (uint8_t)kNfaNoExc;
  for (uint32_t i = 0; i < m; ++i) {
    if (!is_exc[i]) continue;
    NfaExc X{};
    X.follow_u = exc_free[i];
    std::vector<std::pair<uint32_t, U128>> g;
    for (auto& ce : cond_edges[i]) {
      bool placed = false;
      for (auto& x : g)
        if (x.first == ce.first) {
          set_bit(x.second, ce.second);
          placed = true;
        }
      if (!placed) {
        if (g.size() >= kNfaExcCond) return false;
        g.push_back({ce.first, U128{0, 0}});
        set_bit(g.back().second, ce.second);
      }
    }
    X.n_c = (uint32_t)g.size();
    for (uint32_t j = 0; j < X.n_c; ++j) {
      X.r[j] = g[j].first;
      X.follow_c[j] = g[j].second;
    }
    N.exc_of[i] = (uint8_t)excs.size();
    set_bit(N.exc_mask, (int)i);
    excs.push_back(X);
    if (excs.size() > kNfaMaxExc) return false;
  }
  N.n_exc = (uint32_t)excs.size();
  N.n_first_c = (uint32_t)first_c.size();
  for (uint32_t k = 0; k < N.n_first_c; ++k) {
    N.first_r[k] = first_c[k].first;
    N.first_c[k] = first_c[k].second;
  }
  N.n_last_c = (uint32_t)last_c.size();
  for (uint32_t k = 0; k < N.n_last_c; ++k) {
    N.last_r[k] = last_c[k].first;
    N.last_c[k] = last_c[k].second;
  }
  bool cond = N.n_first_c || N.n_last_c;
  for (auto& X : excs) cond |= X.n_c > 0;
  N.has_cond = cond ? 1 : 0;
  // ASCII reach classes: bytes every position treats alike
  std::map<std::pair<uint64_t, uint64_t>, uint32_t> cls_of;
  std::vector<U128> reach;
  for (int ch = 0; ch < 128; ++ch) {
    U128 r{0, 0};
    for (uint32_t i = 0; i < m; ++i)
      if (consumes_ascii(p, p.inst[pcs[i]], ch)) set_bit(r, (int)i);
    auto key = std::make_pair(r.lo, r.hi);
    auto it = cls_of.find(key);
    if (it == cls_of.end()) {
      it = cls_of.emplace(key, (uint32_t)reach.size()).first;
      reach.push_back(r);
    }
    N.cls[ch] = (uint8_t)it->second;
  }
  N.ncls = (uint32_t)reach.size();
  // non-ASCII rune symbols
  N.na_ok = 1;
  for (uint32_t i = 0; i < m; ++i) {
    const Inst& in = p.inst[pcs[i]];
    for (uint32_t j = 0; j + 1 < kDfaRuneSyms; ++j)
      if (consumes_rune(p, in, kSymRune[j])) set_bit(N.reach_sym[j], (int)i);
    const int o = other_runes(p, in);
    if (o == -1) set_bit(N.reach_sym[kDfaRuneSyms - 1], (int)i);
    if (o == 1) N.na_ok = 0;
  }
  N.o_reach = (uint32_t)sizeof(NfaDev);
  N.o_exc = N.o_reach + N.ncls * (uint32_t)sizeof(U128);
  N.bytes = N.o_exc + N.n_exc * (uint32_t)sizeof(NfaExc);
  out->blob.resize(N.bytes);
  memcpy(out->blob.data(), &N, sizeof(N));
  memcpy(out->blob.data() + N.o_reach, reach.data(), reach.size() * sizeof(U128));
  if (!excs.empty()) memcpy(out->blob.data() + N.o_exc, excs.data(), excs.size() * sizeof(NfaExc));
  out->npos = m;
  out->n_exc = N.n_exc;
  out->valid = true;
  return true;
}

int nfa_walk_host(const NfaHost& d, const uint8_t* text, size_t n, size_t s, size_t inj_hi, size_t* me) {
  if (!d.valid || n > 0x7FFFFFFFull || s > n) return 2;
  const NfaDev& N = *(const NfaDev*)d.blob.data();
  const U128* reach = (const U128*)(d.blob.data() + N.o_reach);
  const NfaExc* exc = (const NfaExc*)(d.blob.data() + N.o_exc);
  uint32_t e = 0, steps = 0;
  const int r = N.npos > 64 ? nfa_walk<true>(N, reach, exc, text, (uint32_t)n, (uint32_t)s, (uint32_t)inj_hi, &e, &steps)
                            : nfa_walk<false>(N, reach, exc, text, (uint32_t)n, (uint32_t)s, (uint32_t)inj_hi, &e, &steps);
  if (r == 1) *me = e;
  return r;
}

}  // namespace tsg
