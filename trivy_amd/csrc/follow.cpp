// follow.cpp — per-rule candidate filter ("follow DFA").
//
// An anchor hit h (an occurrence of one of a rule's anchor literals) becomes a
// verification candidate only if some match of the rule's regex can contain
// that occurrence.  This builds, per anchored rule, a small byte DFA that
// decides a NECESSARY condition for that, reading text forward from h:
//
//   Q_h  = NFA states that can be active at h in a run started at any s with
//          [s,h) over the anchor alphabet and h-s <= off_max (gre::Anchor);
//   run  = the NFA state-set from Q_h over text[h..], empty-width assertions
//          treated as satisfied;  a set holding MATCH -> ACCEPT (absorbing),
//          the empty set -> DEAD (reject).
//
// Every real match m=[s,e) containing the literal at h drives the set to
// MATCH by e, so it is ACCEPTed: the filter only ever drops hits that cannot
// anchor a match, and k_verify's leftmost-first FindAll (scanner.go:97-163)
// stays exact (DESIGN.md "Anchors").  Over-approximations that keep it sound:
// bytes >= 0x80 ACCEPT (runes / invalid UTF-8 are left to the exact VM),
// subset construction capped in states (overflow -> ACCEPT), and the device
// walk capped at kFollowDepth bytes (-> ACCEPT).
#include <algorithm>
#include <map>
#include <vector>

#include "engine.h"

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

bool consumes_some_nonascii(const gre::Prog& p, const Inst& in) {
  switch (in.op) {
    case gre::I_RUNE: return p.classes[in.arg].nranges > 0;
    case gre::I_RUNE1: return in.arg >= 128;
    case gre::I_ANY:
    case gre::I_ANYNL: return true;
  }
  return false;
}

bool is_consuming(const Inst& in) {
  return in.op == gre::I_RUNE || in.op == gre::I_RUNE1 || in.op == gre::I_ANY || in.op == gre::I_ANYNL;
}

struct SetBuilder {
  const gre::Prog& p;
  std::vector<uint8_t> seen;
  explicit SetBuilder(const gre::Prog& prog) : p(prog), seen(prog.inst.size(), 0) {}

  // epsilon closure of pc into (consuming pcs, match flag)
  void add(uint32_t pc0, std::vector<uint32_t>* out, bool* match) {
    std::vector<uint32_t> stk{pc0};
    while (!stk.empty()) {
      uint32_t pc = stk.back();
      stk.pop_back();
      if (pc == 0 || pc >= p.inst.size() || seen[pc]) continue;
      seen[pc] = 1;
      const Inst& in = p.inst[pc];
      switch (in.op) {
        case gre::I_MATCH: *match = true; break;
        case gre::I_ALT:
          stk.push_back(in.arg);
          stk.push_back(in.out);
          break;
        case gre::I_CAP:
        case gre::I_EMPTY:  // assertion assumed satisfiable (over-approximation)
        case gre::I_NOP: stk.push_back(in.out); break;
        default:
          if (is_consuming(in)) out->push_back(pc);
      }
    }
  }
  void reset() { std::fill(seen.begin(), seen.end(), 0); }
};

// Q_h: closure of start, then alphabet steps (lengths 1..off_max).
void anchor_entry(const gre::Compiled& c, SetBuilder& sb, std::vector<uint32_t>* qp, bool* qmatch) {
  const gre::Prog& p = c.prog;
  const gre::Anchor& a = c.anchor;
  std::vector<uint32_t>& q = *qp;
  sb.add(p.start, &q, qmatch);
  bool alpha_hi = false;
  for (int b = 128; b < 256; ++b) alpha_hi |= a.alpha.has(b);
  for (uint32_t k = 0; k < a.off_max && !*qmatch; ++k) {
    const size_t before = q.size();
    std::vector<uint32_t> nxt;
    for (uint32_t pc : q) {
      const Inst& in = p.inst[pc];
      bool step = false;
      for (int ch = 0; ch < 128 && !step; ++ch) step = a.alpha.has(ch) && consumes_ascii(p, in, ch);
      if (!step && alpha_hi) step = consumes_some_nonascii(p, in);
      if (step) nxt.push_back(in.out);
    }
    for (uint32_t pc : nxt) sb.add(pc, &q, qmatch);  // `seen` keeps q duplicate-free
    if (q.size() == before) break;  // fixpoint
  }
}

inline uint32_t fold_col(int b) { return (uint32_t)((b & 0x1F) | ((b >> 1) & 0x20)); }

// The fold-special runes: a file holding one (C4B0 / C5BF / E284AA) is
// flagged by k_fold_special and scanned whole for every rule (k_full_jobs),
// its anchor hits dropped — so the scan automaton may assume they are absent.
inline bool fold_special_rune(uint32_t r) { return r == 0x130 || r == 0x17F || r == 0x212A; }

// Can `in` consume a non-ASCII rune other than the fold-special ones?
bool consumes_other_nonascii(const gre::Prog& p, const Inst& in) {
  switch (in.op) {
    case gre::I_RUNE: {
      const gre::ClassDesc& cd = p.classes[in.arg];
      for (uint32_t k = 0; k < cd.nranges; ++k) {
        const uint32_t lo = p.ranges[cd.range_off + 2 * k], hi = p.ranges[cd.range_off + 2 * k + 1];
        for (uint32_t r = lo; r <= hi; ++r)
          if (!fold_special_rune(r)) return true;
      }
      return false;
    }
    case gre::I_RUNE1: return in.arg >= 128 && !fold_special_rune(in.arg);
    case gre::I_ANY:
    case gre::I_ANYNL: return true;
  }
  return false;
}

}  // namespace

// Column sets that every match of the rule must show right after an
// occurrence of anchor literal `lit` (for the scan automaton: a pattern
// "literal + classes" fires far less often than the bare literal — e.g.
// twilio's `SK` followed by two hex digits instead of every "sk" in text).
// Position j's set is the 6-bit fold columns (k_scan_fast's fold6) of every
// ASCII byte some NFA state alive there consumes; extension stops at the
// first position where a non-ASCII rune could be consumed (its bytes alias
// arbitrary columns), where a match may already have ended, or where the set
// is every column.  Sound like build_follow: assertions count as satisfied and
// the alive set is a union over all paths.
std::vector<uint64_t> follow_ext(const gre::Compiled& c, const gre::Lit& lit, int max_ext) {
  std::vector<uint64_t> cols;
  const gre::Prog& p = c.prog;
  if (!c.anchor.valid || p.inst.empty() || p.start == 0 || max_ext <= 0) return cols;
  SetBuilder sb(p);
  std::vector<uint32_t> q;
  bool m = false;
  anchor_entry(c, sb, &q, &m);
  if (m) return cols;
  auto step = [&](const std::vector<uint32_t>& from, const bool* bytes, std::vector<uint32_t>* to) {
    sb.reset();
    to->clear();
    bool mm = false;
    for (uint32_t pc : from) {
      const Inst& in = p.inst[pc];
      bool any = false;
      for (int ch = 0; ch < 128 && !any; ++ch) any = bytes[ch] && consumes_ascii(p, in, ch);
      if (any) sb.add(in.out, to, &mm);
    }
    return mm;
  };
  std::vector<uint32_t> nx;
  for (size_t k = 0; k < lit.lower.size(); ++k) {
    bool bytes[128] = {false};
    const unsigned char lo = (unsigned char)lit.lower[k], rq = (unsigned char)lit.req[k];
    if (lo >= 0x80) return cols;
    if (rq) {
      bytes[rq & 0x7F] = true;
    } else {
      bytes[lo] = true;
      if (lo >= 'a' && lo <= 'z') bytes[lo - 32] = true;
    }
    if (step(q, bytes, &nx)) return cols;  // a match can end inside the literal
    q.swap(nx);
    if (q.empty()) return cols;
  }
  for (int j = 0; j < max_ext; ++j) {
    bool bytes[128] = {false};
    uint64_t mask = 0;
    for (uint32_t pc : q) {
      const Inst& in = p.inst[pc];
      if (consumes_other_nonascii(p, in)) return cols;
      for (int ch = 0; ch < 128; ++ch)
        if (consumes_ascii(p, in, ch)) {
          bytes[ch] = true;
          mask |= 1ull << fold_col(ch);
        }
    }
    if (mask == ~0ull || mask == 0) return cols;
    cols.push_back(mask);
    if (step(q, bytes, &nx)) return cols;  // a match may end here: nothing after is required
    q.swap(nx);
    if (q.empty()) return cols;
  }
  return cols;
}

bool build_follow(const gre::Compiled& c, FollowDfa* out) {
  *out = FollowDfa{};
  const gre::Prog& p = c.prog;
  if (!c.anchor.valid || p.inst.empty() || p.start == 0) return false;
  SetBuilder sb(p);
  std::vector<uint32_t> q;
  bool qmatch = false;
  anchor_entry(c, sb, &q, &qmatch);
  if (qmatch) return false;  // a match can end right at h: nothing to filter
  std::sort(q.begin(), q.end());
  // ---- byte classes over ASCII: bytes accepted by the same consuming insts
  std::vector<uint32_t> cons;
  for (uint32_t pc = 0; pc < p.inst.size(); ++pc)
    if (is_consuming(p.inst[pc])) cons.push_back(pc);
  std::map<std::vector<uint8_t>, int> sig_cls;
  std::vector<int> cls_rep;
  for (int ch = 0; ch < 128; ++ch) {
    std::vector<uint8_t> sig(cons.size());
    for (size_t i = 0; i < cons.size(); ++i) sig[i] = consumes_ascii(p, p.inst[cons[i]], ch);
    auto it = sig_cls.find(sig);
    int k;
    if (it == sig_cls.end()) {
      k = (int)cls_rep.size();
      sig_cls[sig] = k;
      cls_rep.push_back(ch);
    } else {
      k = it->second;
    }
    out->cls[ch] = (uint8_t)k;
  }
  const uint32_t K = (uint32_t)cls_rep.size();
  if (K > 255) return false;
  // ---- subset construction: 0 = DEAD, 1 = ACCEPT, 2 = start
  std::map<std::vector<uint32_t>, uint16_t> ids;
  std::vector<std::vector<uint32_t>> sets(3);
  sets[2] = q;
  ids[q] = 2;
  std::vector<uint16_t> delta(3 * K, 0);
  for (uint32_t k = 0; k < K; ++k) delta[1 * K + k] = 1;
  for (size_t s = 2; s < sets.size(); ++s) {
    for (uint32_t k = 0; k < K; ++k) {
      const int ch = cls_rep[k];
      sb.reset();
      std::vector<uint32_t> nxt;
      bool m = false;
      for (uint32_t pc : sets[s]) {
        const Inst& in = p.inst[pc];
        if (consumes_ascii(p, in, ch)) sb.add(in.out, &nxt, &m);
      }
      uint16_t t;
      if (m) {
        t = 1;
      } else if (nxt.empty()) {
        t = 0;
      } else {
        std::sort(nxt.begin(), nxt.end());
        auto it = ids.find(nxt);
        if (it != ids.end()) {
          t = it->second;
        } else if (sets.size() >= kFollowMaxStates) {
          t = 1;  // state budget exhausted: accept (sound)
        } else {
          t = (uint16_t)sets.size();
          ids[nxt] = t;
          sets.push_back(nxt);
          delta.resize(sets.size() * K, 0);
        }
      }
      delta[s * K + k] = t;
    }
  }
  out->delta = std::move(delta);
  out->ncls = K;
  out->nstates = (uint32_t)sets.size();
  out->valid = true;
  return true;
}

bool follow_accepts(const FollowDfa& f, const uint8_t* text, size_t n, size_t h) {
  if (!f.valid) return true;
  uint32_t st = 2;
  for (uint32_t i = 0; i < kFollowDepth; ++i) {
    if (h + i >= n) return false;
    const uint8_t c = text[h + i];
    if (c >= 0x80) return true;
    st = f.delta[(size_t)st * f.ncls + f.cls[c]];
    if (st < 2) return st == 1;
  }
  return true;
}

}  // namespace tsg
