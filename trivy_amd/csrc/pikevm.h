// pikevm.h — leftmost-first Pike VM over Go-decoded runes, callable from
// host and gfx950 device code.  One VM instance per lane: its thread lists
// live in a caller-provided scratch slice (HBM on the device).
//
// Semantics restate go1.22 regexp/exec.go (machine.match / step / add) as
// driven by Regexp.FindAllIndex / FindAllSubmatchIndex / MatchString in
// pkg/fanal/secret/scanner.go:107,125,166,202,211,259:
//   * runes decoded like utf8.DecodeRune (each invalid byte = U+FFFD, width 1)
//   * a new lowest-priority thread is started at every rune position until
//     a match is found; a MATCH cuts all lower-priority threads
//   * empty-width context from the rune before / after the position.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gre_prog.h"

namespace gre {

// Positions: uint32_t for files below 4 GiB (every hot path), uint64_t for the
// jobs of longer files (the engine instantiates the search twice).  Only the
// text length fixes the type; the other positions convert to it.
template <class T>
struct Ident {
  typedef T type;
};
template <class Pos>
struct SlotOf {  // signed capture slot of a position type (-1 = unset)
  typedef int32_t type;
};
template <>
struct SlotOf<uint64_t> {
  typedef int64_t type;
};
template <>
struct SlotOf<unsigned long long> {
  typedef int64_t type;
};

__host__ __device__ inline int is_word_rune(int r) {
  return (r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_';
}

// utf8.DecodeRune. Returns rune, sets *w (0 at end of text -> rune -1).
template <class Pos>
__host__ __device__ inline int decode_rune(const uint8_t* s, Pos n, typename Ident<Pos>::type i, uint32_t* w) {
  if (i >= n) {
    *w = 0;
    return -1;
  }
  uint32_t c0 = s[i];
  if (c0 < 0x80) {
    *w = 1;
    return (int)c0;
  }
  uint32_t need, lo = 0x80, hi = 0xBF;
  if (c0 >= 0xC2 && c0 <= 0xDF) {
    need = 2;
  } else if (c0 >= 0xE0 && c0 <= 0xEF) {
    need = 3;
    if (c0 == 0xE0) lo = 0xA0;
    if (c0 == 0xED) hi = 0x9F;
  } else if (c0 >= 0xF0 && c0 <= 0xF4) {
    need = 4;
    if (c0 == 0xF0) lo = 0x90;
    if (c0 == 0xF4) hi = 0x8F;
  } else {
    *w = 1;
    return 0xFFFD;
  }
  if (i + need > n) {
    *w = 1;
    return 0xFFFD;
  }
  uint32_t c1 = s[i + 1];
  if (c1 < lo || c1 > hi) {
    *w = 1;
    return 0xFFFD;
  }
  if (need == 2) {
    *w = 2;
    return (int)(((c0 & 0x1F) << 6) | (c1 & 0x3F));
  }
  uint32_t c2 = s[i + 2];
  if (c2 < 0x80 || c2 > 0xBF) {
    *w = 1;
    return 0xFFFD;
  }
  if (need == 3) {
    *w = 3;
    return (int)(((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (c2 & 0x3F));
  }
  uint32_t c3 = s[i + 3];
  if (c3 < 0x80 || c3 > 0xBF) {
    *w = 1;
    return 0xFFFD;
  }
  *w = 4;
  return (int)(((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((c2 & 0x3F) << 6) | (c3 & 0x3F));
}

// True if byte offset i is the start of a rune in the canonical decoding
// from offset 0 (i.e. not inside a valid multi-byte sequence).
template <class Pos>
__host__ __device__ inline bool is_rune_start(const uint8_t* s, Pos n, typename Ident<Pos>::type i) {
  if (i == 0 || i >= n) return true;
  if ((s[i] & 0xC0) != 0x80) return true;
  Pos lim = i >= 3 ? i - 3 : 0;
  for (Pos q = i; q-- > lim;) {
    if ((s[q] & 0xC0) != 0x80) {
      uint32_t w;
      decode_rune(s, n, q, &w);
      return q + w <= i;
    }
  }
  return true;  // only continuation bytes before: each is its own RuneError
}

__host__ __device__ inline uint8_t empty_ctx(int r1, int r2) {
  uint8_t op = kNoWordBoundary;
  if (r1 < 0) op |= kBeginText | kBeginLine;
  if (r1 == '\n') op |= kBeginLine;
  if (r2 < 0) op |= kEndText | kEndLine;
  if (r2 == '\n') op |= kEndLine;
  if (is_word_rune(r1) != is_word_rune(r2)) op ^= (kWordBoundary | kNoWordBoundary);
  return op;
}

// Context rune before position i for empty-width ops: only '\n' and ASCII
// word-ness matter, and DecodeLastRune yields a non-ASCII rune (or
// RuneError) whenever the previous byte is >= 0x80.
template <class Pos>
__host__ __device__ inline int prev_ctx_rune(const uint8_t* s, Pos i) {
  if (i == 0) return -1;
  uint8_t b = s[i - 1];
  return b < 0x80 ? (int)b : 0xFFFD;
}

__host__ __device__ inline bool class_match(const ProgView& p, uint32_t ci, int r) {
  const ClassDesc& c = p.classes[ci];
  if (r < 128) return (c.ascii[r >> 5] >> (r & 31)) & 1;
  const uint32_t* rg = p.ranges + c.range_off;  // sorted, disjoint [lo, hi] pairs
  uint32_t lo = 0, hi = c.nranges;
  while (lo < hi) {  // first range whose hi >= r (Unicode tables run to hundreds of ranges)
    const uint32_t m = (lo + hi) / 2;
    if ((uint32_t)r > rg[2 * m + 1]) lo = m + 1;
    else hi = m;
  }
  return lo < c.nranges && (uint32_t)r >= rg[2 * lo];
}

__host__ __device__ inline bool inst_consumes(const Inst& in, const ProgView& p, int r) {
  switch (in.op) {
    case I_RUNE: return r >= 0 && class_match(p, in.arg, r);
    case I_RUNE1: return r >= 0 && (uint32_t)r == in.arg;
    case I_ANY: return r >= 0;
    case I_ANYNL: return r >= 0 && r != '\n';
  }
  return false;
}

// Scratch for one VM: sized by ninst (and ncap for the capture VM).  The
// position arrays hold Pos / SlotOf<Pos> entries: sized for the widest
// instantiation the owner runs (8 bytes on the device, 4 in the host VM).
struct VmScratch {
  uint16_t* sparse[2];  // [ninst]
  uint16_t* dense[2];   // [ninst] visited pcs in priority order
  void* start[2];       // Pos [ninst] thread start offset (whole-match VM)
  uint16_t* stack;      // [ninst + 1]
  void* caps[2];        // Slot [ninst * ncap]  (capture VM only)
  void* cur;            // Slot [ncap]          (capture VM only)
  void* capstack;       // Slot [2 * ninst + 2] (capture VM only)
};

template <class Pos>
struct Queue {
  typedef typename SlotOf<Pos>::type Slot;
  uint16_t* sparse;
  uint16_t* dense;
  Pos* start;
  Slot* caps;
  uint32_t n;
};

template <class Pos>
__host__ __device__ inline bool q_has(const Queue<Pos>& q, uint32_t pc) {
  uint32_t j = q.sparse[pc];
  return j < q.n && q.dense[j] == pc;
}

// Go's machine.add for the whole-match VM: follow empty transitions from pc
// in priority order, recording every visited pc.
template <class Pos>
__host__ __device__ inline void vm_add(const ProgView& p, Queue<Pos>& q, uint16_t* stack, uint32_t pc0,
                                       Pos st, uint8_t ctx) {
  uint32_t sp = 0;
  stack[sp++] = (uint16_t)pc0;
  while (sp) {
    uint32_t pc = stack[--sp];
    for (;;) {
      if (pc == 0 || q_has(q, pc)) break;
      uint32_t j = q.n++;
      q.sparse[pc] = (uint16_t)j;
      q.dense[j] = (uint16_t)pc;
      q.start[j] = st;
      const Inst in = p.inst[pc];
      if (in.op == I_ALT) {
        stack[sp++] = (uint16_t)in.arg;
        pc = in.out;
        continue;
      }
      if (in.op == I_EMPTY) {
        if ((in.empty & ~ctx) == 0) {
          pc = in.out;
          continue;
        }
        break;
      }
      if (in.op == I_NOP || in.op == I_CAP) {
        pc = in.out;
        continue;
      }
      break;  // consuming instruction or MATCH: a thread parks here
    }
  }
}

// Leftmost-first search from pos0 (a rune boundary) over text[0..n).  New
// start threads are only added at positions <= start_limit.  On success sets
// [*ms, *me) and returns true.  If first_only, returns at the first MATCH
// reached (MatchString semantics: any match).
template <class Pos>
__host__ __device__ inline bool vm_search(const ProgView& p, const uint8_t* text, Pos n,
                                          typename Ident<Pos>::type pos0, typename Ident<Pos>::type start_limit,
                                          bool first_only, VmScratch& sc, Pos* ms, Pos* me) {
  Queue<Pos> q[2] = {{sc.sparse[0], sc.dense[0], (Pos*)sc.start[0], nullptr, 0},
                     {sc.sparse[1], sc.dense[1], (Pos*)sc.start[1], nullptr, 0}};
  int cur = 0;
  bool matched = false;
  uint32_t w = 0, w1 = 0;
  int r = decode_rune(text, n, pos0, &w);
  int r1 = -1;
  if (r >= 0) r1 = decode_rune(text, n, pos0 + w, &w1);
  uint8_t ctx = empty_ctx(prev_ctx_rune(text, pos0), r);
  Pos pos = pos0;
  for (;;) {
    Queue<Pos>& runq = q[cur];
    Queue<Pos>& nextq = q[cur ^ 1];
    if (runq.n == 0) {
      if (matched || pos > start_limit) break;
    }
    if (!matched && pos <= start_limit) vm_add(p, runq, sc.stack, p.start, pos, ctx);
    uint8_t nctx = empty_ctx(r, r1);
    nextq.n = 0;
    for (uint32_t j = 0; j < runq.n; ++j) {
      const Inst in = p.inst[runq.dense[j]];
      if (in.op == I_MATCH) {
        *ms = runq.start[j];
        *me = pos;
        matched = true;
        if (first_only) return true;
        break;  // cut lower-priority threads
      }
      if (inst_consumes(in, p, r)) vm_add(p, nextq, sc.stack, in.out, runq.start[j], nctx);
    }
    runq.n = 0;
    if (w == 0) break;
    pos += w;
    r = r1;
    w = w1;
    if (r >= 0) r1 = decode_rune(text, n, pos + w, &w1);
    else r1 = -1;
    ctx = nctx;
    cur ^= 1;
  }
  return matched;
}

// ---- capture VM (FindAllSubmatchIndex) -----------------------------------

template <class Pos>
__host__ __device__ inline void vmc_add(const ProgView& p, Queue<Pos>& q, VmScratch& sc, uint32_t pc0,
                                        Pos pos, uint8_t ctx) {
  typedef typename SlotOf<Pos>::type Slot;
  // stack entries: pc (tag 0) or capture restore (slot, old) (tag 1)
  const uint32_t ncap = p.ncap;
  Slot* cs = (Slot*)sc.capstack;
  Slot* scur = (Slot*)sc.cur;
  uint32_t sp = 0;
  cs[sp++] = (Slot)pc0;
  cs[sp++] = -1;  // tag -1 = pc entry
  while (sp) {
    Slot tag = cs[--sp];
    Slot val = cs[--sp];
    if (tag >= 0) {  // restore cap[tag] = val
      scur[tag] = val;
      continue;
    }
    uint32_t pc = (uint32_t)val;
    for (;;) {
      if (pc == 0 || q_has(q, pc)) break;
      uint32_t j = q.n++;
      q.sparse[pc] = (uint16_t)j;
      q.dense[j] = (uint16_t)pc;
      const Inst in = p.inst[pc];
      if (in.op == I_ALT) {
        cs[sp++] = (Slot)in.arg;
        cs[sp++] = -1;
        pc = in.out;
        continue;
      }
      if (in.op == I_EMPTY) {
        if ((in.empty & ~ctx) == 0) {
          pc = in.out;
          continue;
        }
        break;
      }
      if (in.op == I_NOP) {
        pc = in.out;
        continue;
      }
      if (in.op == I_CAP) {
        if (in.arg < ncap) {
          cs[sp++] = scur[in.arg];
          cs[sp++] = (Slot)in.arg;  // restore after the subtree
          scur[in.arg] = (Slot)pos;
        }
        pc = in.out;
        continue;
      }
      Slot* dst = q.caps + (size_t)j * ncap;
      for (uint32_t k = 0; k < ncap; ++k) dst[k] = scur[k];
      break;
    }
  }
}

// Anchored capture run at position s (must be a rune boundary): returns the
// leftmost-first match starting at s with all capture slots in caps_out.
template <class Pos>
__host__ __device__ inline bool vm_captures(const ProgView& p, const uint8_t* text, Pos n,
                                            typename Ident<Pos>::type s, VmScratch& sc,
                                            typename SlotOf<Pos>::type* caps_out) {
  typedef typename SlotOf<Pos>::type Slot;
  const uint32_t ncap = p.ncap;
  Slot* scur = (Slot*)sc.cur;
  Queue<Pos> q[2] = {{sc.sparse[0], sc.dense[0], nullptr, (Slot*)sc.caps[0], 0},
                     {sc.sparse[1], sc.dense[1], nullptr, (Slot*)sc.caps[1], 0}};
  int cur = 0;
  bool matched = false;
  uint32_t w = 0, w1 = 0;
  int r = decode_rune(text, n, s, &w);
  int r1 = -1;
  if (r >= 0) r1 = decode_rune(text, n, s + w, &w1);
  uint8_t ctx = empty_ctx(prev_ctx_rune(text, s), r);
  Pos pos = s;
  for (uint32_t k = 0; k < ncap; ++k) caps_out[k] = -1;
  bool first = true;
  for (;;) {
    Queue<Pos>& runq = q[cur];
    Queue<Pos>& nextq = q[cur ^ 1];
    if (runq.n == 0 && !first) break;
    if (first) {
      for (uint32_t k = 0; k < ncap; ++k) scur[k] = -1;
      scur[0] = (Slot)pos;
      vmc_add(p, runq, sc, p.start, pos, ctx);
      first = false;
    }
    uint8_t nctx = empty_ctx(r, r1);
    nextq.n = 0;
    for (uint32_t j = 0; j < runq.n; ++j) {
      const Inst in = p.inst[runq.dense[j]];
      Slot* tc = runq.caps + (size_t)j * ncap;
      if (in.op == I_MATCH) {
        for (uint32_t k = 0; k < ncap; ++k) caps_out[k] = tc[k];
        caps_out[1] = (Slot)pos;
        matched = true;
        break;
      }
      if (inst_consumes(in, p, r)) {
        for (uint32_t k = 0; k < ncap; ++k) scur[k] = tc[k];
        vmc_add(p, nextq, sc, in.out, pos + w, nctx);
      }
    }
    runq.n = 0;
    if (w == 0) break;
    pos += w;
    r = r1;
    w = w1;
    if (r >= 0) r1 = decode_rune(text, n, pos + w, &w1);
    else r1 = -1;
    ctx = nctx;
    cur ^= 1;
  }
  return matched;
}

}  // namespace gre
