// Instruction program shared by the host compiler (gre.cpp) and the Pike VM
// (pikevm.h) that runs on gfx950.  Layout mirrors the *meaning* of Go's
// regexp/syntax Prog (Inst{Op,Out,Arg}) — leftmost-first priority is carried
// by ALT.out (preferred) vs ALT.arg — but is our own flat POD encoding.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace gre {

enum InstOp : uint8_t {
  I_FAIL = 0,   // pc 0 is always FAIL (a patched-to-0 edge means "no path")
  I_MATCH = 1,
  I_RUNE = 2,   // arg = class index
  I_RUNE1 = 3,  // arg = rune
  I_ANY = 4,    // any rune (?s).
  I_ANYNL = 5,  // any rune except '\n'
  I_ALT = 6,    // out preferred, arg second
  I_CAP = 7,    // arg = capture slot
  I_EMPTY = 8,  // empty = required EmptyOp flags
  I_NOP = 9,
};

// Go's syntax.EmptyOp bits.
enum : uint8_t {
  kBeginLine = 1,
  kEndLine = 2,
  kBeginText = 4,
  kEndText = 8,
  kWordBoundary = 16,
  kNoWordBoundary = 32,
};

struct Inst {
  uint8_t op;
  uint8_t empty;
  uint16_t vis;  // bit-state visited-row index (join points only), kNoVis elsewhere
  uint32_t out;
  uint32_t arg;
};

// Only join points (instructions with two or more reachable predecessors,
// plus the start) get a visited row in the capture backtracker: every cycle
// passes through one, and an instruction with a single predecessor is reached
// at most as often as that predecessor (bounded), so memoising the join points
// keeps the search polynomial with a fraction of the (pc, pos) bits.
constexpr uint16_t kNoVis = 0xFFFF;

struct ClassDesc {
  uint32_t ascii[4];   // membership bitmap for runes < 128
  uint32_t range_off;  // into Prog::ranges (pairs lo,hi), runes >= 128 only
  uint32_t nranges;
};

struct Prog {
  std::vector<Inst> inst;
  std::vector<ClassDesc> classes;
  std::vector<uint32_t> ranges;
  uint32_t start = 0;
  int ncap = 2;                         // 2 * (number of groups + 1)
  uint32_t nvis = 0;                    // instructions with a visited row (Inst::vis)
  std::vector<std::string> cap_names;   // index = group number; [0] = ""
};

// Flat, pointer-based view (host or device memory).
struct ProgView {
  const Inst* inst;
  const ClassDesc* classes;
  const uint32_t* ranges;
  uint32_t ninst;
  uint32_t start;
  uint32_t ncap;
  uint32_t nvis;
};

}  // namespace gre
