// dfa.cpp — per-rule anchored leftmost-first DFA for k_verify.
//
// Go's FindAllIndex (scanner.go:107 -> regexp.go allMatches) returns, from a
// search position, the leftmost start with a match and, at that start, the
// match Go's backtracking priority prefers.  k_verify already knows the
// permitted starts (anchor windows), so it needs, per start s, the
// leftmost-first match END of the regex anchored at s.  This builds that
// automaton RE2-style: a DFA state is the ORDERED list of NFA threads (the
// consuming instructions a Pike VM would hold, in priority order), cut after
// MATCH — exactly the queue regexp/exec.go's machine keeps, minus the threads
// its `break` on MATCH drops.  Walking it: every state with `match` set moves
// the match end to the current position (a higher-priority thread matched);
// the walk stops when the list is empty.
//
// Symbols: the ASCII byte classes, then five rune symbols for the decoded
// non-ASCII runes (utf8.DecodeRune, an invalid byte is U+FFFD of width 1):
// U+212A K, U+017F ſ, U+0130 İ (the runes Go's case rules tie to ASCII
// letters), U+FFFD, and "any other non-ASCII rune" -- the last only when
// every consuming instruction treats all those runes alike (na_ok; ASCII
// classes, (?i) letters, negated ASCII classes and `.` do), else a walk that
// meets such a rune is left to the Pike VM.  The only empty-width assertions
// are ^ / $ without (?m) (kBeginText / kEndText): BeginText is a start-state
// choice (s == 0), and EndText only matters when the last rune of the text
// is consumed, so every transition carries an "end match" bit computed with
// EndText satisfied.
#include <algorithm>
#include <map>
#include <vector>

#include "engine.h"
#include "pikevm.h"

namespace tsg {
namespace {

using gre::Inst;

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

// The rune symbols after the ASCII classes (DfaHost::sym_base + j).
constexpr uint32_t kSymRune[kDfaRuneSyms - 1] = {0x212A, 0x17F, 0x130, 0xFFFD};

bool class_has(const gre::Prog& p, const gre::ClassDesc& cd, uint32_t r) {
  for (uint32_t k = 0; k < cd.nranges; ++k)
    if (p.ranges[cd.range_off + 2 * k] <= r && r <= p.ranges[cd.range_off + 2 * k + 1]) return true;
  return false;
}

// Non-ASCII runes other than kSymRune (surrogates never decode): how many an
// instruction consumes -- 0 (none), -1 (all), or some (not one symbol).
int other_runes(const gre::Prog& p, const Inst& in) {
  auto in_dom = [](uint64_t r) { return r >= 0x80 && r <= 0x10FFFF && !(r >= 0xD800 && r <= 0xDFFF); };
  uint64_t dom = (0x10FFFF - 0x80 + 1) - 0x800 - (sizeof(kSymRune) / sizeof(kSymRune[0]));
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
      uint64_t n = 0;
      for (uint32_t k = 0; k < cd.nranges; ++k) {
        uint64_t lo = std::max<uint64_t>(p.ranges[cd.range_off + 2 * k], 0x80);
        uint64_t hi = std::min<uint64_t>(p.ranges[cd.range_off + 2 * k + 1], 0x10FFFF);
        if (lo > hi) continue;
        n += hi - lo + 1;
        const uint64_t slo = std::max<uint64_t>(lo, 0xD800), shi = std::min<uint64_t>(hi, 0xDFFF);
        if (slo <= shi) n -= shi - slo + 1;
        for (uint32_t r : kSymRune)
          if (r >= lo && r <= hi && in_dom(r)) --n;
      }
      return n == 0 ? 0 : n == dom ? -1 : 1;
    }
  }
  return 0;
}

// Does `in` consume rune symbol j (kSymRune[j], or any other non-ASCII rune)?
bool consumes_sym(const gre::Prog& p, const Inst& in, uint32_t j) {
  if (j + 1 == kDfaRuneSyms) return other_runes(p, in) == -1;
  const uint32_t r = kSymRune[j];
  switch (in.op) {
    case gre::I_RUNE: return class_has(p, p.classes[in.arg], r);
    case gre::I_RUNE1: return in.arg == r;
    case gre::I_ANY:
    case gre::I_ANYNL: return true;
  }
  return false;
}

bool is_consuming(const Inst& in) {
  return in.op == gre::I_RUNE || in.op == gre::I_RUNE1 || in.op == gre::I_ANY || in.op == gre::I_ANYNL;
}

// machine.add: follow empty transitions from pc in priority order (ALT: out
// before arg), parking consuming instructions in `list`; a MATCH sets
// *matched and cuts everything after it.
struct Closure {
  const gre::Prog& p;
  std::vector<uint8_t> seen;
  explicit Closure(const gre::Prog& prog) : p(prog), seen(prog.inst.size(), 0) {}
  void reset() { std::fill(seen.begin(), seen.end(), 0); }
  void add(uint32_t pc0, uint8_t ctx, std::vector<uint32_t>* list, bool* matched) {
    std::vector<uint32_t> stk{pc0};
    while (!stk.empty() && !*matched) {
      uint32_t pc = stk.back();
      stk.pop_back();
      while (!*matched) {
        if (pc == 0 || pc >= p.inst.size() || seen[pc]) break;
        seen[pc] = 1;
        const Inst& in = p.inst[pc];
        if (in.op == gre::I_ALT) {
          stk.push_back(in.arg);
          pc = in.out;
          continue;
        }
        if (in.op == gre::I_EMPTY) {
          if ((in.empty & ~ctx) == 0) {
            pc = in.out;
            continue;
          }
          break;
        }
        if (in.op == gre::I_NOP || in.op == gre::I_CAP) {
          pc = in.out;
          continue;
        }
        if (in.op == gre::I_MATCH) {
          *matched = true;
          break;
        }
        if (is_consuming(in)) list->push_back(pc);
        break;
      }
    }
  }
};

}  // namespace

bool build_dfa(const gre::Compiled& c, DfaHost* out) {
  *out = DfaHost{};
  const gre::Prog& p = c.prog;
  if (p.inst.empty() || p.start == 0) return false;
  for (const Inst& in : p.inst)
    if (in.op == gre::I_EMPTY && (in.empty & ~(gre::kBeginText | gre::kEndText))) return false;
  // ASCII byte classes (bytes every consuming instruction treats alike)
  std::vector<uint32_t> cons;
  for (uint32_t pc = 0; pc < p.inst.size(); ++pc)
    if (is_consuming(p.inst[pc])) cons.push_back(pc);
  std::map<std::vector<uint8_t>, int> sig_cls;
  std::vector<int> rep;
  for (int ch = 0; ch < 128; ++ch) {
    std::vector<uint8_t> sig(cons.size());
    for (size_t i = 0; i < cons.size(); ++i) sig[i] = consumes_ascii(p, p.inst[cons[i]], ch);
    auto it = sig_cls.find(sig);
    if (it == sig_cls.end()) {
      it = sig_cls.emplace(sig, (int)rep.size()).first;
      rep.push_back(ch);
    }
    out->cls[ch] = (uint8_t)it->second;
  }
  const uint32_t KA = (uint32_t)rep.size();  // ASCII classes; rune symbols follow
  const uint32_t K = KA + kDfaRuneSyms;
  if (KA > 128) return false;
  out->sym_base = KA;
  out->na_ok = true;
  for (uint32_t pc : cons) out->na_ok &= other_runes(p, p.inst[pc]) != 1;
  auto consumes = [&](const Inst& in, uint32_t k) {
    return k < KA ? consumes_ascii(p, in, rep[k]) : consumes_sym(p, in, k - KA);
  };
  // states: 0 = dead; lists are keyed with their match flag
  std::map<std::pair<std::vector<uint32_t>, bool>, uint16_t> ids;
  std::vector<std::vector<uint32_t>> lists(1);
  std::vector<uint8_t> match(1, 0);
  Closure cl(p);
  auto intern = [&](std::vector<uint32_t>& l, bool m, bool* overflow) -> uint16_t {
    if (l.empty() && !m) return 0;
    auto key = std::make_pair(l, m);
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    if (lists.size() >= kDfaMaxStates) {
      *overflow = true;
      return 0;
    }
    const uint16_t id = (uint16_t)lists.size();
    ids.emplace(key, id);
    lists.push_back(l);
    match.push_back(m ? 1 : 0);
    return id;
  };
  bool overflow = false;
  for (int bt = 0; bt < 2; ++bt) {
    std::vector<uint32_t> l;
    bool m = false;
    cl.reset();
    cl.add(p.start, bt ? gre::kBeginText : 0, &l, &m);
    out->start[bt] = intern(l, m, &overflow);
  }
  std::vector<uint16_t> delta;
  for (size_t s = 1; s < lists.size() && !overflow; ++s) {
    delta.resize(lists.size() * K, 0);
    for (uint32_t k = 0; k < K; ++k) {
      std::vector<uint32_t> nl;
      bool m = false;
      cl.reset();
      for (uint32_t pc : lists[s])
        if (consumes(p.inst[pc], k)) cl.add(p.inst[pc].out, 0, &nl, &m);
      // the same step landing on the last rune of the text: EndText holds
      std::vector<uint32_t> el;
      bool em = false;
      cl.reset();
      for (uint32_t pc : lists[s])
        if (consumes(p.inst[pc], k)) cl.add(p.inst[pc].out, gre::kEndText, &el, &em);
      const uint16_t t = intern(nl, m, &overflow);
      delta.resize(lists.size() * K, 0);
      delta[s * K + k] = (uint16_t)(t | (em ? 0x8000 : 0));
    }
  }
  if (overflow) return false;
  delta.resize(lists.size() * K, 0);
  // bit 14: the target state is a match state (saves the walk a dependent load)
  for (auto& v : delta)
    if (match[v & kDfaStateMask]) v |= 0x4000;
  // first-byte filter: a start position whose byte kills both start states
  // (and does not end a match as the last byte) cannot match
  for (int c = 0; c < 128; ++c)
    for (int bt = 0; bt < 2; ++bt) {
      const uint16_t e = delta[(size_t)out->start[bt] * K + out->cls[c]];
      if ((e & kDfaStateMask) || (e & 0x8000) || match[out->start[bt]]) out->first[c >> 5] |= 1u << (c & 31);
    }
  out->delta = std::move(delta);
  out->match = std::move(match);
  out->ncls = K;
  out->nstates = (uint32_t)lists.size();
  out->valid = true;
  return true;
}

// Symbol of the rune at text[q] (q < n, text[q] >= 0x80) and its width;
// -1 when the DFA cannot take it (a non-ASCII rune its classes tell apart).
int dfa_rune_sym(const DfaHost& d, const uint8_t* text, size_t n, size_t q, uint32_t* w) {
  const int r = gre::decode_rune(text, (uint32_t)n, (uint32_t)q, w);
  for (uint32_t j = 0; j + 1 < kDfaRuneSyms; ++j)
    if ((uint32_t)r == kSymRune[j]) return (int)(d.sym_base + j);
  return d.na_ok ? (int)(d.sym_base + kDfaRuneSyms - 1) : -1;
}

// Host mirror of the device walk (tests / diagnostics): 1 = match [s, *me),
// 0 = none, 2 = not decidable here (a rune the DFA cannot take, or s at the end).
int dfa_anchored(const DfaHost& d, const uint8_t* text, size_t n, size_t s, size_t* me) {
  if (!d.valid || s >= n) return 2;
  uint32_t st = d.start[s == 0 ? 1 : 0];
  int64_t last = d.match[st] ? (int64_t)s : -1;
  for (size_t q = s; q < n && st;) {
    const uint8_t c = text[q];
    uint32_t w = 1, k = d.cls[c & 0x7F];
    if (c >= 0x80) {
      const int sym = dfa_rune_sym(d, text, n, q, &w);
      if (sym < 0) return 2;
      k = (uint32_t)sym;
    }
    const uint16_t e = d.delta[(size_t)st * d.ncls + k];
    if (q + w == n) {
      if (e & 0x8000) last = (int64_t)n;
      break;
    }
    st = e & kDfaStateMask;
    q += w;
    if (e & 0x4000) last = (int64_t)q;
  }
  if (last < 0) return 0;
  *me = (size_t)last;
  return 1;
}

}  // namespace tsg
