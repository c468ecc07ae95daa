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

__host__ __device__ inline int is_word_rune(int r) {
  return (r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_';
}

// utf8.DecodeRune. Returns rune, sets *w (0 at end of text -> rune -1).
__host__ __device__ inline int decode_rune(const uint8_t* s, uint32_t n, uint32_t i, uint32_t* w) {
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
__host__ __device__ inline bool is_rune_start(const uint8_t* s, uint32_t n, uint32_t i) {
  if (i == 0 || i >= n) return true;
  if ((s[i] & 0xC0) != 0x80) return true;
  uint32_t lim = i >= 3 ? i - 3 : 0;
  for (uint32_t q = i; q-- > lim;) {
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
__host__ __device__ inline int prev_ctx_rune(const uint8_t* s, uint32_t i) {
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

// Scratch for one VM: sized by ninst (and ncap for the capture VM).
struct VmScratch {
  uint16_t* sparse[2];  // [ninst]
  uint16_t* dense[2];   // [ninst] visited pcs in priority order
  uint32_t* start[2];   // [ninst] thread start offset (whole-match VM)
  uint16_t* stack;      // [ninst + 1]
  int32_t* caps[2];     // [ninst * ncap]  (capture VM only)
  int32_t* cur;         // [ncap]          (capture VM only)
  int32_t* capstack;    // [2 * ninst + 2] (capture VM only)
};

struct Queue {
  uint16_t* sparse;
  uint16_t* dense;
  uint32_t* start;
  int32_t* caps;
  uint32_t n;
};

__host__ __device__ inline bool q_has(const Queue& q, uint32_t pc) {
  uint32_t j = q.sparse[pc];
  return j < q.n && q.dense[j] == pc;
}

// Go's machine.add for the whole-match VM: follow empty transitions from pc
// in priority order, recording every visited pc.
__host__ __device__ inline void vm_add(const ProgView& p, Queue& q, uint16_t* stack, uint32_t pc0,
                                       uint32_t st, uint8_t ctx) {
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
__host__ __device__ inline bool vm_search(const ProgView& p, const uint8_t* text, uint32_t n,
                                          uint32_t pos0, uint32_t start_limit, bool first_only,
                                          VmScratch& sc, uint32_t* ms, uint32_t* me) {
  Queue q[2] = {{sc.sparse[0], sc.dense[0], sc.start[0], nullptr, 0},
                {sc.sparse[1], sc.dense[1], sc.start[1], nullptr, 0}};
  int cur = 0;
  bool matched = false;
  uint32_t w = 0, w1 = 0;
  int r = decode_rune(text, n, pos0, &w);
  int r1 = -1;
  if (r >= 0) r1 = decode_rune(text, n, pos0 + w, &w1);
  uint8_t ctx = empty_ctx(prev_ctx_rune(text, pos0), r);
  uint32_t pos = pos0;
  for (;;) {
    Queue& runq = q[cur];
    Queue& nextq = q[cur ^ 1];
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

__host__ __device__ inline void vmc_add(const ProgView& p, Queue& q, VmScratch& sc, uint32_t pc0,
                                        uint32_t pos, uint8_t ctx) {
  // stack entries: pc (tag 0) or capture restore (slot, old) (tag 1)
  const uint32_t ncap = p.ncap;
  int32_t* cs = sc.capstack;
  uint32_t sp = 0;
  cs[sp++] = (int32_t)pc0;
  cs[sp++] = -1;  // tag -1 = pc entry
  while (sp) {
    int32_t tag = cs[--sp];
    int32_t val = cs[--sp];
    if (tag >= 0) {  // restore cap[tag] = val
      sc.cur[tag] = val;
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
        cs[sp++] = (int32_t)in.arg;
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
          cs[sp++] = sc.cur[in.arg];
          cs[sp++] = (int32_t)in.arg;  // restore after the subtree
          sc.cur[in.arg] = (int32_t)pos;
        }
        pc = in.out;
        continue;
      }
      int32_t* dst = q.caps + (size_t)j * ncap;
      for (uint32_t k = 0; k < ncap; ++k) dst[k] = sc.cur[k];
      break;
    }
  }
}

// Anchored capture run at position s (must be a rune boundary): returns the
// leftmost-first match starting at s with all capture slots in caps_out.
__host__ __device__ inline bool vm_captures(const ProgView& p, const uint8_t* text, uint32_t n,
                                            uint32_t s, VmScratch& sc, int32_t* caps_out) {
  const uint32_t ncap = p.ncap;
  Queue q[2] = {{sc.sparse[0], sc.dense[0], nullptr, sc.caps[0], 0},
                {sc.sparse[1], sc.dense[1], nullptr, sc.caps[1], 0}};
  int cur = 0;
  bool matched = false;
  uint32_t w = 0, w1 = 0;
  int r = decode_rune(text, n, s, &w);
  int r1 = -1;
  if (r >= 0) r1 = decode_rune(text, n, s + w, &w1);
  uint8_t ctx = empty_ctx(prev_ctx_rune(text, s), r);
  uint32_t pos = s;
  for (uint32_t k = 0; k < ncap; ++k) caps_out[k] = -1;
  bool first = true;
  for (;;) {
    Queue& runq = q[cur];
    Queue& nextq = q[cur ^ 1];
    if (runq.n == 0 && !first) break;
    if (first) {
      for (uint32_t k = 0; k < ncap; ++k) sc.cur[k] = -1;
      sc.cur[0] = (int32_t)pos;
      vmc_add(p, runq, sc, p.start, pos, ctx);
      first = false;
    }
    uint8_t nctx = empty_ctx(r, r1);
    nextq.n = 0;
    for (uint32_t j = 0; j < runq.n; ++j) {
      const Inst in = p.inst[runq.dense[j]];
      int32_t* tc = runq.caps + (size_t)j * ncap;
      if (in.op == I_MATCH) {
        for (uint32_t k = 0; k < ncap; ++k) caps_out[k] = tc[k];
        caps_out[1] = (int32_t)pos;
        matched = true;
        break;
      }
      if (inst_consumes(in, p, r)) {
        for (uint32_t k = 0; k < ncap; ++k) sc.cur[k] = tc[k];
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
