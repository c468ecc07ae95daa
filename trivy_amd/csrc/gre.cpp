// gre.cpp — Go RE2 syntax parser, Go-priority program compiler and anchor
// analysis.  See gre.h.  Semantics follow go1.22 regexp/syntax (parse.go,
// simplify.go, compile.go) as used by pkg/fanal/secret/scanner.go; the code is
// an independent implementation (recursive descent + patch lists).
#include "gre.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>

#include "gre_fold_table.h"
#include "gre_unicode_tables.h"

namespace gre {

uint32_t simple_fold(uint32_t r) {
  int lo = 0, hi = kFoldOrbitLen;
  while (lo < hi) {
    int m = (lo + hi) / 2;
    if (kFoldOrbit[m][0] < r) lo = m + 1; else hi = m;
  }
  if (lo < kFoldOrbitLen && kFoldOrbit[lo][0] == r) return kFoldOrbit[lo][1];
  return r;
}

namespace {

constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr uint32_t kRuneError = 0xFFFD;

enum NOp { NO_NOMATCH, NO_EMPTY, NO_LIT, NO_CLASS, NO_ANYNL, NO_ANY, NO_ASSERT, NO_CAP,
           NO_STAR, NO_PLUS, NO_QUEST, NO_REPEAT, NO_CONCAT, NO_ALT };

struct Node {
  NOp op = NO_EMPTY;
  bool nongreedy = false;
  uint32_t rune = 0;
  std::vector<uint32_t> cls;  // sorted, merged [lo,hi] pairs
  uint8_t empty = 0;
  int cap = 0;
  int min = 0, max = 0;
  std::vector<Node*> sub;
};

struct Flags {
  bool i = false, m = false, s = false, U = false;
};

struct SyntaxError {
  std::string msg;
};

// ---------------------------------------------------------------- classes --
void clean_class(std::vector<uint32_t>& c) {
  std::vector<std::pair<uint32_t, uint32_t>> v;
  for (size_t k = 0; k + 1 < c.size(); k += 2) v.push_back({c[k], c[k + 1]});
  std::sort(v.begin(), v.end());
  std::vector<uint32_t> out;
  for (auto& p : v) {
    if (!out.empty() && p.first <= out.back() + 1) {
      out.back() = std::max(out.back(), p.second);
    } else {
      out.push_back(p.first);
      out.push_back(p.second);
    }
  }
  c.swap(out);
}

void append_range(std::vector<uint32_t>& c, uint32_t lo, uint32_t hi) {
  c.push_back(lo);
  c.push_back(hi);
}

// appendFoldedRange: add [lo,hi] and the simple-fold orbit of every member.
void append_folded_range(std::vector<uint32_t>& c, uint32_t lo, uint32_t hi) {
  append_range(c, lo, hi);
  // walk orbit-table entries inside [lo,hi]
  int a = 0, b = kFoldOrbitLen;
  while (a < b) {
    int m = (a + b) / 2;
    if (kFoldOrbit[m][0] < lo) a = m + 1; else b = m;
  }
  for (int k = a; k < kFoldOrbitLen && kFoldOrbit[k][0] <= hi; ++k) {
    uint32_t r = kFoldOrbit[k][0];
    for (uint32_t f = simple_fold(r); f != r; f = simple_fold(f)) append_range(c, f, f);
  }
}

std::vector<uint32_t> negate_class(const std::vector<uint32_t>& c) {
  std::vector<uint32_t> out;
  uint32_t next = 0;
  for (size_t k = 0; k + 1 < c.size(); k += 2) {
    if (c[k] > next) append_range(out, next, c[k] - 1);
    next = c[k + 1] + 1;
  }
  if (next <= kMaxRune) append_range(out, next, kMaxRune);
  return out;
}

struct PerlGroup {
  const char* name;
  std::vector<uint32_t> ranges;
};

std::vector<uint32_t> perl_class(char c) {
  switch (c) {
    case 'd': return {'0', '9'};
    case 's': return {'\t', '\n', '\f', '\r', ' ', ' '};
    case 'w': return {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'};
  }
  return {};
}

bool posix_class(const std::string& name, std::vector<uint32_t>* out) {
  static const struct { const char* n; std::vector<uint32_t> r; } tbl[] = {
      {"alnum", {'0', '9', 'A', 'Z', 'a', 'z'}},
      {"alpha", {'A', 'Z', 'a', 'z'}},
      {"ascii", {0, 0x7f}},
      {"blank", {'\t', '\t', ' ', ' '}},
      {"cntrl", {0, 0x1f, 0x7f, 0x7f}},
      {"digit", {'0', '9'}},
      {"graph", {'!', '~'}},
      {"lower", {'a', 'z'}},
      {"print", {' ', '~'}},
      {"punct", {'!', '/', ':', '@', '[', '`', '{', '~'}},
      {"space", {'\t', '\r', ' ', ' '}},
      {"upper", {'A', 'Z'}},
      {"word", {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}},
      {"xdigit", {'0', '9', 'A', 'F', 'a', 'f'}},
  };
  for (auto& e : tbl) {
    if (name == e.n) {
      *out = e.r;
      return true;
    }
  }
  return false;
}

// unicodeTable (regexp/syntax parse.go): "Any", then unicode.Categories, then
// unicode.Scripts (tables: gre_unicode_tables.h, Unicode 15.0 as in Go 1.22).
bool unicode_table(const std::string& name, std::vector<uint32_t>* out) {
  out->clear();
  if (name == "Any") {
    *out = {0, kMaxRune};
    return true;
  }
  for (uint32_t t = 0; t < kUniTableCount; ++t) {
    if (name != kUniTables[t].name) continue;
    for (uint32_t k = 0; k < kUniTables[t].n; ++k) {
      out->push_back(kUniRanges[kUniTables[t].off + k][0]);
      out->push_back(kUniRanges[kUniTables[t].off + k][1]);
    }
    return true;
  }
  return false;
}

// ----------------------------------------------------------------- parser --
class Parser {
 public:
  explicit Parser(const std::string& s) : p_(s) {}

  Node* parse() {
    Flags f;
    Node* n = parse_alt(f);
    if (i_ != p_.size()) throw SyntaxError{"unexpected ): `" + p_ + "`"};
    return n;
  }
  int ncap() const { return ncap_; }
  std::vector<std::string> names() const { return names_; }

 private:
  const std::string& p_;
  size_t i_ = 0;
  int ncap_ = 0;
  std::vector<std::string> names_{""};
  std::vector<std::unique_ptr<Node>> arena_;

 public:
  std::vector<std::unique_ptr<Node>>& arena() { return arena_; }

 private:
  Node* make(NOp op) {
    arena_.push_back(std::make_unique<Node>());
    arena_.back()->op = op;
    return arena_.back().get();
  }
  bool eof() const { return i_ >= p_.size(); }
  char peek(size_t k = 0) const { return i_ + k < p_.size() ? p_[i_ + k] : '\0'; }

  uint32_t next_rune() {
    // decode one UTF-8 rune from the pattern (Go rejects invalid UTF-8)
    unsigned char c = p_[i_];
    if (c < 0x80) { ++i_; return c; }
    int n = (c >= 0xF0) ? 4 : (c >= 0xE0) ? 3 : (c >= 0xC0) ? 2 : 0;
    if (n == 0 || i_ + n > p_.size()) throw SyntaxError{"invalid UTF-8"};
    uint32_t r = c & (0x7F >> n);
    for (int k = 1; k < n; ++k) {
      unsigned char cc = p_[i_ + k];
      if ((cc & 0xC0) != 0x80) throw SyntaxError{"invalid UTF-8"};
      r = (r << 6) | (cc & 0x3F);
    }
    i_ += n;
    return r;
  }

  Node* literal(uint32_t r, const Flags& f) {
    if (f.i && simple_fold(r) != r) {
      Node* n = make(NO_CLASS);
      append_folded_range(n->cls, r, r);
      clean_class(n->cls);
      return n;
    }
    Node* n = make(NO_LIT);
    n->rune = r;
    return n;
  }

  Node* class_node(std::vector<uint32_t> c) {
    clean_class(c);
    Node* n = make(NO_CLASS);
    n->cls = std::move(c);
    if (n->cls.empty()) n->op = NO_NOMATCH;
    return n;
  }

  Node* parse_alt(Flags f) {  // f: group-scoped flags (shared by branches)
    std::vector<Node*> br;
    br.push_back(parse_concat(f));
    while (peek() == '|' && !eof()) {
      ++i_;
      br.push_back(parse_concat(f));
    }
    if (br.size() == 1) return br[0];
    Node* n = make(NO_ALT);
    n->sub = br;
    return n;
  }

  // Try to parse "{n}", "{n,}", "{n,m}" at i_. Returns false (no consume)
  // if the text is not a valid repeat, in which case '{' is a literal.
  bool parse_repeat_spec(int* mn, int* mx, size_t* len) {
    size_t j = i_ + 1;
    auto num = [&](int* v) -> bool {
      size_t s = j;
      long x = 0;
      while (j < p_.size() && isdigit((unsigned char)p_[j])) {
        x = x * 10 + (p_[j] - '0');
        if (x > 100000) x = 100000;
        ++j;
      }
      if (j == s) return false;
      *v = (int)x;
      return true;
    };
    if (!num(mn)) return false;
    if (j < p_.size() && p_[j] == ',') {
      ++j;
      if (j < p_.size() && p_[j] == '}') {
        *mx = -1;
      } else if (!num(mx)) {
        return false;
      }
    } else {
      *mx = *mn;
    }
    if (j >= p_.size() || p_[j] != '}') return false;
    *len = j + 1 - i_;
    return true;
  }

  Node* parse_concat(Flags& f) {
    std::vector<Node*> items;
    bool last_repeat = false;
    while (!eof() && peek() != '|' && peek() != ')') {
      char c = peek();
      if (c == '*' || c == '+' || c == '?' || c == '{') {
        int mn = 0, mx = 0;
        size_t len = 1;
        NOp op;
        if (c == '{') {
          if (!parse_repeat_spec(&mn, &mx, &len)) {
            // literal '{'
            ++i_;
            items.push_back(literal('{', f));
            last_repeat = false;
            continue;
          }
          if (mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx))
            throw SyntaxError{"invalid repeat count"};
          op = NO_REPEAT;
        } else {
          op = c == '*' ? NO_STAR : c == '+' ? NO_PLUS : NO_QUEST;
        }
        if (items.empty()) throw SyntaxError{"missing argument to repetition operator"};
        if (last_repeat) throw SyntaxError{"invalid nested repetition operator"};
        i_ += len;
        bool ng = false;
        if (peek() == '?' && !eof()) {
          ++i_;
          ng = true;
        }
        if (f.U) ng = !ng;
        Node* n = make(op);
        n->nongreedy = ng;
        n->min = mn;
        n->max = mx;
        n->sub.push_back(items.back());
        items.back() = n;
        last_repeat = true;
        continue;
      }
      last_repeat = false;
      if (c == '(') {
        Node* g = parse_group(f);
        if (g) items.push_back(g);
        continue;
      }
      if (c == '[') {
        items.push_back(parse_class(f));
        continue;
      }
      if (c == '.') {
        ++i_;
        items.push_back(make(f.s ? NO_ANY : NO_ANYNL));
        continue;
      }
      if (c == '^') {
        ++i_;
        Node* n = make(NO_ASSERT);
        n->empty = f.m ? kBeginLine : kBeginText;
        items.push_back(n);
        continue;
      }
      if (c == '$') {
        ++i_;
        Node* n = make(NO_ASSERT);
        n->empty = f.m ? kEndLine : kEndText;
        items.push_back(n);
        continue;
      }
      if (c == '\\') {
        parse_escape(f, items);
        continue;
      }
      items.push_back(literal(next_rune(), f));
    }
    if (items.size() == 1) return items[0];
    Node* n = make(items.empty() ? NO_EMPTY : NO_CONCAT);
    n->sub = items;
    return n;
  }

  void apply_flags(const std::string& spec, Flags* f) {
    bool neg = false, sawneg = false, any = false;
    for (char c : spec) {
      if (c == '-') {
        if (sawneg) throw SyntaxError{"invalid or unsupported Perl syntax"};
        neg = sawneg = true;
        any = false;
        continue;
      }
      bool v = !neg;
      if (c == 'i') f->i = v;
      else if (c == 'm') f->m = v;
      else if (c == 's') f->s = v;
      else if (c == 'U') f->U = v;
      else throw SyntaxError{"invalid or unsupported Perl syntax"};
      any = true;
    }
    if (sawneg && !any) throw SyntaxError{"invalid or unsupported Perl syntax"};
  }

  Node* parse_group(Flags& f) {
    ++i_;  // (
    if (peek() == '?') {
      if (peek(1) == 'P' && peek(2) == '<' ) { i_ += 3; return named_group(f); }
      if (peek(1) == '<') { i_ += 2; return named_group(f); }
      size_t j = i_ + 1;
      while (j < p_.size() && strchr("imsU-", p_[j]) && p_[j]) ++j;
      if (j >= p_.size() || (p_[j] != ')' && p_[j] != ':'))
        throw SyntaxError{"invalid or unsupported Perl syntax"};
      std::string spec = p_.substr(i_ + 1, j - i_ - 1);
      if (p_[j] == ')') {
        if (spec.empty()) throw SyntaxError{"invalid or unsupported Perl syntax"};
        apply_flags(spec, &f);
        i_ = j + 1;
        return nullptr;
      }
      Flags inner = f;
      apply_flags(spec, &inner);
      i_ = j + 1;
      Node* body = parse_alt(inner);
      if (peek() != ')' || eof()) throw SyntaxError{"missing closing )"};
      ++i_;
      return body;
    }
    int cap = ++ncap_;
    names_.push_back("");
    Node* body = parse_alt(f);
    if (peek() != ')' || eof()) throw SyntaxError{"missing closing )"};
    ++i_;
    Node* n = make(NO_CAP);
    n->cap = cap;
    n->sub.push_back(body);
    return n;
  }

  Node* named_group(Flags& f) {
    size_t end = p_.find('>', i_);
    if (end == std::string::npos) throw SyntaxError{"invalid named capture"};
    std::string name = p_.substr(i_, end - i_);
    if (name.empty()) throw SyntaxError{"invalid named capture"};
    for (char c : name)
      if (!(isalnum((unsigned char)c) || c == '_')) throw SyntaxError{"invalid named capture"};
    i_ = end + 1;
    int cap = ++ncap_;
    names_.push_back(name);
    Node* body = parse_alt(f);
    if (peek() != ')' || eof()) throw SyntaxError{"missing closing )"};
    ++i_;
    Node* n = make(NO_CAP);
    n->cap = cap;
    n->sub.push_back(body);
    return n;
  }

  std::vector<uint32_t> group_ranges(const std::vector<uint32_t>& g, bool neg, const Flags& f) {
    std::vector<uint32_t> tmp;
    if (f.i) {
      for (size_t k = 0; k + 1 < g.size(); k += 2) append_folded_range(tmp, g[k], g[k + 1]);
    } else {
      tmp = g;
    }
    clean_class(tmp);
    return neg ? negate_class(tmp) : tmp;
  }

  // \p{Name}, \pN, \P{Name}, \p{^Name} (parse.go parseUnicodeClass), i_ just
  // past the 'p' / 'P'.  Under (?i) the table's simple-fold closure joins it
  // before any negation (Go's unicode.FoldCategory / FoldScript additions).
  std::vector<uint32_t> unicode_class(bool neg, const Flags& f) {
    const size_t start = i_ - 2;  // the backslash
    std::string name;
    if (peek() != '{' || eof()) {
      const size_t b = i_;
      if (!eof()) next_rune();
      name = p_.substr(b, i_ - b);
    } else {
      const size_t end = p_.find('}', i_);
      if (end == std::string::npos)
        throw SyntaxError{"invalid character class range: `" + p_.substr(start) + "`"};
      name = p_.substr(i_ + 1, end - i_ - 1);
      i_ = end + 1;
    }
    const std::string seq = p_.substr(start, i_ - start);
    if (!name.empty() && name[0] == '^') {
      neg = !neg;
      name = name.substr(1);
    }
    std::vector<uint32_t> tab;
    if (!unicode_table(name, &tab)) throw SyntaxError{"invalid character class range: `" + seq + "`"};
    if (f.i) {
      std::vector<uint32_t> folded;
      for (size_t k = 0; k + 1 < tab.size(); k += 2) append_folded_range(folded, tab[k], tab[k + 1]);
      tab.swap(folded);
    }
    clean_class(tab);
    return neg ? negate_class(tab) : tab;
  }

  // Simple escapes shared by class and non-class context; returns rune.
  uint32_t simple_escape(char c) {
    switch (c) {
      case 'a': return 7;
      case 'f': return 12;
      case 't': return 9;
      case 'n': return 10;
      case 'r': return 13;
      case 'v': return 11;
    }
    if (c == 'x') {
      if (peek() == '{') {
        size_t end = p_.find('}', i_);
        if (end == std::string::npos || end == i_ + 1) throw SyntaxError{"invalid escape sequence"};
        uint32_t v = 0;
        for (size_t k = i_ + 1; k < end; ++k) {
          if (!isxdigit((unsigned char)p_[k])) throw SyntaxError{"invalid escape sequence"};
          v = v * 16 + (isdigit((unsigned char)p_[k]) ? p_[k] - '0' : (tolower(p_[k]) - 'a' + 10));
          if (v > kMaxRune) throw SyntaxError{"invalid escape sequence"};
        }
        i_ = end + 1;
        return v;
      }
      if (i_ + 2 > p_.size() || !isxdigit((unsigned char)p_[i_]) || !isxdigit((unsigned char)p_[i_ + 1]))
        throw SyntaxError{"invalid escape sequence"};
      uint32_t v = 0;
      for (int k = 0; k < 2; ++k) {
        char h = p_[i_ + k];
        v = v * 16 + (isdigit((unsigned char)h) ? h - '0' : (tolower(h) - 'a' + 10));
      }
      i_ += 2;
      return v;
    }
    if (c >= '0' && c <= '7') {
      // \1-\7 alone are backreferences (unsupported); octal needs a 0 or a 2nd digit
      if (c != '0' && !(peek() >= '0' && peek() <= '7')) throw SyntaxError{"invalid escape sequence"};
      uint32_t v = c - '0';
      for (int k = 0; k < 2 && peek() >= '0' && peek() <= '7' && !eof(); ++k) {
        v = v * 8 + (peek() - '0');
        ++i_;
      }
      return v;
    }
    if ((unsigned char)c < 0x80 && !isalnum((unsigned char)c)) return (unsigned char)c;
    throw SyntaxError{std::string("invalid escape sequence: `\\") + c + "`"};
  }

  void parse_escape(const Flags& f, std::vector<Node*>& items) {
    ++i_;  // backslash
    if (eof()) throw SyntaxError{"trailing backslash at end of expression"};
    char c = p_[i_++];
    switch (c) {
      case 'A': case 'z': case 'b': case 'B': {
        Node* n = make(NO_ASSERT);
        n->empty = c == 'A' ? kBeginText : c == 'z' ? kEndText : c == 'b' ? kWordBoundary : kNoWordBoundary;
        items.push_back(n);
        return;
      }
      case 'd': case 's': case 'w': case 'D': case 'S': case 'W': {
        items.push_back(class_node(group_ranges(perl_class((char)tolower(c)), isupper((unsigned char)c), f)));
        return;
      }
      case 'p': case 'P':
        items.push_back(class_node(unicode_class(c == 'P', f)));
        return;
      case 'Q': {
        size_t end = p_.find("\\E", i_);
        size_t stop = end == std::string::npos ? p_.size() : end;
        while (i_ < stop) items.push_back(literal(next_rune(), f));
        i_ = end == std::string::npos ? p_.size() : end + 2;
        return;
      }
      case 'C':
        throw SyntaxError{"invalid escape sequence: `\\C`"};
    }
    items.push_back(literal(simple_escape(c), f));
  }

  // One class element: returns false if it was a perl/posix group appended to out.
  bool class_char(const Flags& f, std::vector<uint32_t>& out, uint32_t* r) {
    if (peek() == '\\') {
      ++i_;
      if (eof()) throw SyntaxError{"trailing backslash at end of expression"};
      char c = p_[i_++];
      if (strchr("dswDSW", c)) {
        auto g = group_ranges(perl_class((char)tolower(c)), isupper((unsigned char)c), f);
        out.insert(out.end(), g.begin(), g.end());
        return false;
      }
      if (c == 'p' || c == 'P') {
        auto g = unicode_class(c == 'P', f);
        out.insert(out.end(), g.begin(), g.end());
        return false;
      }
      *r = simple_escape(c);
      return true;
    }
    *r = next_rune();
    return true;
  }

  Node* parse_class(const Flags& f) {
    ++i_;  // [
    bool neg = false;
    if (peek() == '^' && !eof()) {
      neg = true;
      ++i_;
    }
    std::vector<uint32_t> cls;
    bool first = true;
    while (true) {
      if (eof()) throw SyntaxError{"missing closing ]"};
      if (peek() == ']' && !first) {
        ++i_;
        break;
      }
      first = false;
      if (peek() == '[' && peek(1) == ':') {
        size_t end = p_.find(":]", i_ + 2);
        if (end != std::string::npos) {
          std::string name = p_.substr(i_ + 2, end - i_ - 2);
          bool pneg = !name.empty() && name[0] == '^';
          if (pneg) name = name.substr(1);
          std::vector<uint32_t> g;
          if (!posix_class(name, &g)) throw SyntaxError{"invalid character class range"};
          auto gg = group_ranges(g, pneg, f);
          cls.insert(cls.end(), gg.begin(), gg.end());
          i_ = end + 2;
          continue;
        }
      }
      uint32_t lo;
      if (!class_char(f, cls, &lo)) continue;
      uint32_t hi = lo;
      if (peek() == '-' && peek(1) != ']' && i_ + 1 < p_.size()) {
        ++i_;
        std::vector<uint32_t> dummy;
        if (!class_char(f, dummy, &hi)) throw SyntaxError{"invalid character class range"};
        if (hi < lo) throw SyntaxError{"invalid character class range"};
      }
      if (f.i) append_folded_range(cls, lo, hi); else append_range(cls, lo, hi);
    }
    clean_class(cls);
    if (neg) cls = negate_class(cls);
    return class_node(cls);
  }
};

// --------------------------------------------------------------- compiler --
struct Frag {
  uint32_t i = 0;                 // 0 = fail
  std::vector<uint32_t> out;      // patch list: (pc<<1)|which
  bool nullable = false;
};

class Compiler {
 public:
  explicit Compiler(Prog* p) : p_(p) {
    p_->inst.clear();
    p_->inst.push_back(Inst{I_FAIL, 0, 0, 0, 0});
  }

  Frag compile(const Node* n) {
    switch (n->op) {
      case NO_NOMATCH: return Frag{};
      case NO_EMPTY: return nop();
      case NO_LIT: return rune1(n->rune);
      case NO_CLASS: return rune_class(n->cls);
      case NO_ANYNL: return simple(I_ANYNL);
      case NO_ANY: return simple(I_ANY);
      case NO_ASSERT: {
        Frag f = inst(I_EMPTY);
        p_->inst[f.i].empty = n->empty;
        f.out = {f.i << 1};
        f.nullable = true;
        return f;
      }
      case NO_CAP: {
        Frag bra = cap(2 * n->cap);
        Frag sub = compile(n->sub[0]);
        Frag ket = cap(2 * n->cap + 1);
        return cat(cat(bra, sub), ket);
      }
      case NO_STAR: return star(compile(n->sub[0]), n->nongreedy);
      case NO_PLUS: return plus(compile(n->sub[0]), n->nongreedy);
      case NO_QUEST: return quest(compile(n->sub[0]), n->nongreedy);
      case NO_REPEAT: return repeat(n);
      case NO_CONCAT: {
        if (n->sub.empty()) return nop();
        Frag f;
        for (size_t k = 0; k < n->sub.size(); ++k) f = k == 0 ? compile(n->sub[k]) : cat(f, compile(n->sub[k]));
        return f;
      }
      case NO_ALT: {
        Frag f;
        bool first = true;
        for (auto* s : n->sub) {
          Frag g = compile(s);
          f = first ? g : alt(f, g);
          first = false;
        }
        return f;
      }
    }
    return Frag{};
  }

  void finish(Frag f) {
    Frag m = inst(I_MATCH);
    patch(f.out, m.i);
    p_->start = f.i;
  }

 private:
  Prog* p_;
  std::vector<std::pair<std::vector<uint32_t>, uint32_t>> class_cache_;

  Frag inst(uint8_t op) {
    Frag f;
    f.i = (uint32_t)p_->inst.size();
    p_->inst.push_back(Inst{op, 0, 0, 0, 0});
    return f;
  }
  void patch(const std::vector<uint32_t>& l, uint32_t target) {
    for (uint32_t e : l) {
      Inst& in = p_->inst[e >> 1];
      if (e & 1) in.arg = target; else in.out = target;
    }
  }
  Frag nop() {
    Frag f = inst(I_NOP);
    f.out = {f.i << 1};
    f.nullable = true;
    return f;
  }
  Frag simple(uint8_t op) {
    Frag f = inst(op);
    f.out = {f.i << 1};
    return f;
  }
  Frag rune1(uint32_t r) {
    Frag f = inst(I_RUNE1);
    p_->inst[f.i].arg = r;
    f.out = {f.i << 1};
    return f;
  }
  Frag rune_class(const std::vector<uint32_t>& cls) {
    uint32_t ci = class_index(cls);
    Frag f = inst(I_RUNE);
    p_->inst[f.i].arg = ci;
    f.out = {f.i << 1};
    return f;
  }
  uint32_t class_index(const std::vector<uint32_t>& cls) {
    for (auto& e : class_cache_)
      if (e.first == cls) return e.second;
    ClassDesc d{};
    d.range_off = (uint32_t)p_->ranges.size();
    for (size_t k = 0; k + 1 < cls.size(); k += 2) {
      uint32_t lo = cls[k], hi = cls[k + 1];
      for (uint32_t r = lo; r <= std::min(hi, 127u); ++r) d.ascii[r >> 5] |= 1u << (r & 31);
      if (hi >= 128) {
        p_->ranges.push_back(std::max(lo, 128u));
        p_->ranges.push_back(hi);
        d.nranges++;
      }
    }
    uint32_t idx = (uint32_t)p_->classes.size();
    p_->classes.push_back(d);
    class_cache_.push_back({cls, idx});
    return idx;
  }
  Frag cap(uint32_t slot) {
    Frag f = inst(I_CAP);
    p_->inst[f.i].arg = slot;
    f.out = {f.i << 1};
    f.nullable = true;
    return f;
  }
  Frag cat(Frag f1, Frag f2) {
    if (f1.i == 0 || f2.i == 0) return Frag{};
    patch(f1.out, f2.i);
    return Frag{f1.i, f2.out, f1.nullable && f2.nullable};
  }
  Frag alt(Frag f1, Frag f2) {
    if (f1.i == 0) return f2;
    if (f2.i == 0) return f1;
    Frag f = inst(I_ALT);
    p_->inst[f.i].out = f1.i;
    p_->inst[f.i].arg = f2.i;
    f.out = f1.out;
    f.out.insert(f.out.end(), f2.out.begin(), f2.out.end());
    f.nullable = f1.nullable || f2.nullable;
    return f;
  }
  Frag quest(Frag f1, bool ng) {
    Frag f = inst(I_ALT);
    f.nullable = true;
    if (ng) {
      p_->inst[f.i].arg = f1.i;
      f.out = {f.i << 1};
    } else {
      p_->inst[f.i].out = f1.i;
      f.out = {(f.i << 1) | 1};
    }
    f.out.insert(f.out.end(), f1.out.begin(), f1.out.end());
    return f;
  }
  Frag loop(Frag f1, bool ng) {
    Frag f = inst(I_ALT);
    if (ng) {
      p_->inst[f.i].arg = f1.i;
      f.out = {f.i << 1};
    } else {
      p_->inst[f.i].out = f1.i;
      f.out = {(f.i << 1) | 1};
    }
    patch(f1.out, f.i);
    return f;
  }
  Frag star(Frag f1, bool ng) {
    if (f1.nullable) return quest(plus(f1, ng), ng);  // golang.org/issue/46123
    return loop(f1, ng);
  }
  Frag plus(Frag f1, bool ng) {
    Frag l = loop(f1, ng);
    return Frag{f1.i, l.out, f1.nullable};
  }
  // simplify.go expansion of x{n,m}
  Frag repeat(const Node* n) {
    const Node* sub = n->sub[0];
    int mn = n->min, mx = n->max;
    bool ng = n->nongreedy;
    if (mn == 0 && mx == 0) return nop();
    if (mx == -1) {
      if (mn == 0) return star(compile(sub), ng);
      if (mn == 1) return plus(compile(sub), ng);
      Frag f;
      for (int k = 0; k < mn - 1; ++k) f = k == 0 ? compile(sub) : cat(f, compile(sub));
      return cat(f, plus(compile(sub), ng));
    }
    if (mn == 1 && mx == 1) return compile(sub);
    Frag prefix;
    bool have_prefix = false;
    for (int k = 0; k < mn; ++k) {
      prefix = have_prefix ? cat(prefix, compile(sub)) : compile(sub);
      have_prefix = true;
    }
    if (mx > mn) {
      // suffix = (x(x(x)?)?)? built inside-out, compiled outside-in so the
      // instruction order is irrelevant; priorities match simplify.go.
      std::function<Frag(int)> nest = [&](int depth) -> Frag {
        // depth counts remaining optional copies (>=1)
        Frag x = compile(sub);
        if (depth == 1) return quest(x, ng);
        return quest(cat(x, nest(depth - 1)), ng);
      };
      Frag suffix = nest(mx - mn);
      return have_prefix ? cat(prefix, suffix) : suffix;
    }
    return have_prefix ? prefix : Frag{};
  }
};

// simplify1's idempotence rule: (?:x*)* == x*, etc.
void simplify(Node* n) {
  for (auto* s : n->sub) simplify(s);
  if ((n->op == NO_STAR || n->op == NO_PLUS || n->op == NO_QUEST) && !n->sub.empty()) {
    Node* s = n->sub[0];
    if (s->op == NO_EMPTY) {
      *n = *s;
      return;
    }
    if (s->op == n->op && s->nongreedy == n->nongreedy) {
      Node copy = *s;
      *n = copy;
    }
  }
}

// ---------------------------------------------------------------- analysis --
constexpr size_t kExactCap = 16;
constexpr size_t kLitMaxLen = 16;

struct A {
  uint32_t minlen = 0, maxlen = 0;
  bool exact = false;
  std::vector<Lit> ex;
  Anchor best;
  Bitmap256 alpha;
  bool nullable = false;
};

uint32_t add_len(uint32_t a, uint32_t b) {
  if (a == kInf || b == kInf) return kInf;
  uint64_t s = (uint64_t)a + b;
  return s >= kInf ? kInf : (uint32_t)s;
}
uint32_t mul_len(uint32_t a, int n) {
  if (n == 0) return 0;
  if (a == kInf) return kInf;
  uint64_t s = (uint64_t)a * (uint64_t)n;
  return s >= kInf ? kInf : (uint32_t)s;
}

int utf8_len(uint32_t r) { return r < 0x80 ? 1 : r < 0x800 ? 2 : r < 0x10000 ? 3 : 4; }

double char_bits(unsigned char lower, unsigned char req) {
  if (lower >= 'a' && lower <= 'z') return req ? 5.5 : 4.2;
  if (lower >= '0' && lower <= '9') return 4.5;
  if (lower == ' ' || lower == '\t') return 3.0;
  if (lower >= 0x80) return 7.0;
  return 5.0;
}

double score_lits(const std::vector<Lit>& lits) {
  if (lits.empty()) return -1e9;
  double mn = 1e9;
  for (auto& l : lits) {
    if (l.lower.empty()) return -1e9;
    double b = 0;
    for (size_t k = 0; k < l.lower.size(); ++k) b += char_bits(l.lower[k], l.req[k]);
    mn = std::min(mn, b);
  }
  return mn - std::log2((double)lits.size());
}

void consider(Anchor* best, const std::vector<Lit>& lits, uint32_t omin, uint32_t omax,
              const Bitmap256& alpha) {
  for (auto& l : lits)
    if (l.lower.empty() || l.lower.size() > kLitMaxLen) return;
  double s = score_lits(lits);
  // Unbounded offsets are located by a backward scan over `alpha`: cheap
  // when alpha stops at word boundaries, line-long when it holds ' ' or '\n'.
  if (omax == kInf) {
    s -= 2.0;
    if (alpha.has('\n')) s -= 30.0;
    if (alpha.has(' ')) s -= 6.0;
  }
  if (!best->valid || s > best->score + 1e-9 ||
      (std::fabs(s - best->score) < 1e-9 && omax < best->off_max)) {
    best->valid = true;
    best->lits = lits;
    best->off_min = omin;
    best->off_max = omax;
    best->alpha = alpha;
    best->score = s;
  }
}

bool product(const std::vector<Lit>& a, const std::vector<Lit>& b, std::vector<Lit>* out) {
  if (a.size() * b.size() > kExactCap) return false;
  out->clear();
  for (auto& x : a)
    for (auto& y : b) {
      Lit z{x.lower + y.lower, x.req + y.req};
      if (z.lower.size() > 64) return false;
      if (std::find(out->begin(), out->end(), z) == out->end()) out->push_back(z);
    }
  return true;
}

void add_unique(std::vector<Lit>* v, const Lit& l) {
  if (std::find(v->begin(), v->end(), l) == v->end()) v->push_back(l);
}

// exact single-char set for a class or literal; false if not representable
bool class_exact(const std::vector<uint32_t>& cls, std::vector<Lit>* out) {
  out->clear();
  bool present[128] = {false};
  for (size_t k = 0; k + 1 < cls.size(); k += 2) {
    for (uint64_t r = cls[k]; r <= cls[k + 1]; ++r) {
      if (r < 128) {
        present[r] = true;
      } else if (r == 0x212A || r == 0x17F) {
        // fold runes: files containing them take the full-scan path
      } else {
        return false;
      }
      if (r - cls[k] > 64) return false;
    }
  }
  for (int c = 0; c < 128; ++c) {
    if (!present[c]) continue;
    if (c >= 'A' && c <= 'Z') {
      if (present[c + 32]) continue;  // handled at the lowercase letter
      add_unique(out, Lit{std::string(1, (char)(c + 32)), std::string(1, (char)c)});
    } else if (c >= 'a' && c <= 'z') {
      bool both = present[c - 32];
      add_unique(out, Lit{std::string(1, (char)c), std::string(1, both ? '\0' : (char)c)});
    } else {
      add_unique(out, Lit{std::string(1, (char)c), std::string(1, '\0')});
    }
  }
  return !out->empty() && out->size() <= 8;
}

void class_lens(const std::vector<uint32_t>& cls, uint32_t* mn, uint32_t* mx, Bitmap256* alpha) {
  uint32_t lo = 4, hi = 0;
  for (size_t k = 0; k + 1 < cls.size(); k += 2) {
    uint32_t a = cls[k], b = cls[k + 1];
    lo = std::min<uint32_t>(lo, utf8_len(a));
    hi = std::max<uint32_t>(hi, utf8_len(b));
    if (a <= kRuneError && kRuneError <= b) lo = 1;  // invalid bytes decode to U+FFFD (width 1)
    for (uint32_t r = a; r <= std::min(b, 127u); ++r) alpha->set((int)r);
    if (b >= 128) alpha->set_range(0x80, 0xFF);
  }
  *mn = cls.empty() ? 0 : lo;
  *mx = hi;
}

A analyze(const Node* n) {
  A a;
  switch (n->op) {
    case NO_NOMATCH:
      a.minlen = a.maxlen = 0;
      return a;
    case NO_EMPTY:
    case NO_ASSERT:
      a.exact = true;
      a.ex = {Lit{"", ""}};
      a.nullable = true;
      return a;
    case NO_LIT: {
      std::vector<uint32_t> cls{n->rune, n->rune};
      class_lens(cls, &a.minlen, &a.maxlen, &a.alpha);
      a.exact = class_exact(cls, &a.ex);
      if (a.exact) consider(&a.best, a.ex, 0, 0, Bitmap256{});
      return a;
    }
    case NO_CLASS: {
      class_lens(n->cls, &a.minlen, &a.maxlen, &a.alpha);
      a.exact = class_exact(n->cls, &a.ex);
      if (a.exact) consider(&a.best, a.ex, 0, 0, Bitmap256{});
      return a;
    }
    case NO_ANYNL:
    case NO_ANY:
      a.minlen = 1;
      a.maxlen = 4;
      a.alpha.set_range(0, 255);
      if (n->op == NO_ANYNL) a.alpha.w[0] &= ~(1ull << '\n');
      return a;
    case NO_CAP:
      return analyze(n->sub[0]);
    case NO_STAR:
    case NO_PLUS:
    case NO_QUEST:
    case NO_REPEAT: {
      A c = analyze(n->sub[0]);
      int mn = n->op == NO_STAR || n->op == NO_QUEST ? 0 : n->op == NO_PLUS ? 1 : n->min;
      int mx = n->op == NO_QUEST ? 1 : (n->op == NO_REPEAT ? n->max : -1);
      a.alpha = c.alpha;
      a.minlen = mul_len(c.minlen, mn);
      a.maxlen = mx < 0 ? (c.maxlen == 0 ? 0 : kInf) : mul_len(c.maxlen, mx);
      a.nullable = mn == 0 || c.nullable;
      if (mn >= 1 && c.best.valid) a.best = c.best;
      if (c.exact) {
        if (mx == mn && mn >= 0) {
          std::vector<Lit> cur{Lit{"", ""}};
          bool ok = true;
          for (int k = 0; k < mn && ok; ++k) {
            std::vector<Lit> nx;
            ok = product(cur, c.ex, &nx);
            cur = nx;
          }
          if (ok) {
            a.exact = true;
            a.ex = cur;
          }
        } else if (mn == 0 && mx == 1) {
          a.exact = true;
          a.ex = c.ex;
          add_unique(&a.ex, Lit{"", ""});
          if (a.ex.size() > kExactCap) a.exact = false;
        }
      }
      if (a.exact) {
        bool nonempty = true;
        for (auto& l : a.ex) nonempty &= !l.lower.empty();
        if (nonempty) consider(&a.best, a.ex, 0, 0, Bitmap256{});
      }
      return a;
    }
    case NO_CONCAT: {
      std::vector<A> ch;
      for (auto* s : n->sub) ch.push_back(analyze(s));
      size_t k = ch.size();
      std::vector<uint32_t> pmin(k + 1, 0), pmax(k + 1, 0);
      std::vector<Bitmap256> palpha(k + 1);
      a.nullable = true;
      for (size_t j = 0; j < k; ++j) {
        pmin[j + 1] = add_len(pmin[j], ch[j].minlen);
        pmax[j + 1] = add_len(pmax[j], ch[j].maxlen);
        palpha[j + 1] = palpha[j];
        palpha[j + 1].merge(ch[j].alpha);
        a.nullable = a.nullable && ch[j].nullable;
      }
      a.minlen = pmin[k];
      a.maxlen = pmax[k];
      a.alpha = palpha[k];
      for (size_t j = 0; j < k; ++j) {
        if (ch[j].best.valid) {
          Bitmap256 al = palpha[j];
          al.merge(ch[j].best.alpha);
          consider(&a.best, ch[j].best.lits, add_len(pmin[j], ch[j].best.off_min),
                   add_len(pmax[j], ch[j].best.off_max), al);
        }
      }
      // windows of consecutive exact children
      for (size_t i = 0; i < k; ++i) {
        if (!ch[i].exact) continue;
        std::vector<Lit> cur{Lit{"", ""}};
        for (size_t j = i; j < k && ch[j].exact; ++j) {
          std::vector<Lit> nx;
          if (!product(cur, ch[j].ex, &nx)) break;
          cur = nx;
          bool ok = true;
          size_t maxl = 0;
          for (auto& l : cur) {
            ok &= !l.lower.empty();
            maxl = std::max(maxl, l.lower.size());
          }
          if (maxl > kLitMaxLen) break;
          if (ok) consider(&a.best, cur, pmin[i], pmax[i], palpha[i]);
        }
      }
      // whole-node exactness
      bool all = true;
      std::vector<Lit> cur{Lit{"", ""}};
      for (size_t j = 0; j < k && all; ++j) {
        std::vector<Lit> nx;
        all = ch[j].exact && product(cur, ch[j].ex, &nx);
        cur = nx;
      }
      if (all) {
        a.exact = true;
        a.ex = cur;
      }
      return a;
    }
    case NO_ALT: {
      std::vector<A> ch;
      for (auto* s : n->sub) ch.push_back(analyze(s));
      a.minlen = kInf;
      a.maxlen = 0;
      bool all_exact = true, all_factor = true;
      std::vector<Lit> ex, fl;
      uint32_t omin = kInf, omax = 0;
      Bitmap256 fal;
      for (auto& c : ch) {
        a.minlen = std::min(a.minlen, c.minlen);
        a.maxlen = (a.maxlen == kInf || c.maxlen == kInf) ? kInf : std::max(a.maxlen, c.maxlen);
        a.alpha.merge(c.alpha);
        a.nullable = a.nullable || c.nullable;
        if (c.exact) {
          for (auto& l : c.ex) add_unique(&ex, l);
        } else {
          all_exact = false;
        }
        if (c.best.valid) {
          for (auto& l : c.best.lits) add_unique(&fl, l);
          omin = std::min(omin, c.best.off_min);
          omax = std::max(omax, c.best.off_max);
          fal.merge(c.best.alpha);
        } else {
          all_factor = false;
        }
      }
      if (all_exact && ex.size() <= kExactCap) {
        a.exact = true;
        a.ex = ex;
        bool nonempty = true;
        for (auto& l : ex) nonempty &= !l.lower.empty();
        if (nonempty) consider(&a.best, ex, 0, 0, Bitmap256{});
      }
      if (all_factor && fl.size() <= 2 * kExactCap) consider(&a.best, fl, omin, omax, fal);
      return a;
    }
  }
  return a;
}

bool has_assert(const Node* n) {
  if (n->op == NO_ASSERT) return true;
  for (auto* s : n->sub)
    if (has_assert(s)) return true;
  return false;
}

}  // namespace


// Capture-group span from the whole match alone (see gre.h GroupSpan).  The
// program is a graph (consuming insts weigh 1 rune, the rest 0); a distance is
// "fixed" when every path has the same rune count, found by propagation in
// which a second, different distance (or a consuming cycle) turns a node into
// "many".  The group's CAP pair must be unique and must dominate every MATCH.
GroupSpan group_span(const Prog& p, uint32_t slot) {
  GroupSpan g;
  const int n = (int)p.inst.size();
  int open = -1, close = -1;
  for (int pc = 0; pc < n; ++pc) {
    const Inst& in = p.inst[pc];
    if (in.op != I_CAP) continue;
    if (in.arg == 2 * slot) {
      if (open >= 0) return g;
      open = pc;
    } else if (in.arg == 2 * slot + 1) {
      if (close >= 0) return g;
      close = pc;
    }
  }
  if (open < 0 || close < 0) return g;
  auto succ = [&](int pc, int* out) -> int {  // successor count, out[0..1]
    const Inst& in = p.inst[pc];
    switch (in.op) {
      case I_FAIL:
      case I_MATCH: return 0;
      case I_ALT: out[0] = (int)in.out; out[1] = (int)in.arg; return 2;
      default: out[0] = (int)in.out; return 1;
    }
  };
  auto weight = [&](int pc) {
    const uint8_t op = p.inst[pc].op;
    return (op == I_RUNE || op == I_RUNE1 || op == I_ANY || op == I_ANYNL) ? 1 : 0;
  };
  // MATCH reachable from start when node `cut` is removed?
  auto reaches_match = [&](int cut) {
    std::vector<uint8_t> seen(n, 0);
    std::vector<int> st{(int)p.start};
    while (!st.empty()) {
      const int pc = st.back();
      st.pop_back();
      if (pc == cut || pc <= 0 || pc >= n || seen[pc]) continue;
      seen[pc] = 1;
      if (p.inst[pc].op == I_MATCH) return true;
      int o[2];
      for (int k = succ(pc, o); k-- > 0;) st.push_back(o[k]);
    }
    return false;
  };
  if (reaches_match(open) || reaches_match(close)) return g;  // the group may not participate
  constexpr int kUnset = -1, kMany = -2;
  // forward: runes from the match start to each node's entry
  std::vector<int> fw(n, kUnset);
  {
    std::vector<int> wl{(int)p.start};
    fw[p.start] = 0;
    while (!wl.empty()) {
      const int pc = wl.back();
      wl.pop_back();
      int o[2];
      const int k = succ(pc, o);
      for (int q = 0; q < k; ++q) {
        const int t = o[q];
        if (t <= 0 || t >= n) continue;
        const int d = fw[pc] == kMany ? kMany : fw[pc] + weight(pc);
        if (fw[t] == kUnset) fw[t] = d;
        else if (fw[t] != d && fw[t] != kMany) fw[t] = kMany;
        else continue;
        wl.push_back(t);
      }
    }
  }
  // backward: runes from each node's entry to the match end
  std::vector<std::vector<int>> pred(n);
  for (int pc = 1; pc < n; ++pc) {
    int o[2];
    for (int k = succ(pc, o); k-- > 0;)
      if (o[k] > 0 && o[k] < n) pred[o[k]].push_back(pc);
  }
  std::vector<int> bw(n, kUnset);
  {
    std::vector<int> wl;
    for (int pc = 1; pc < n; ++pc)
      if (p.inst[pc].op == I_MATCH) {
        bw[pc] = 0;
        wl.push_back(pc);
      }
    while (!wl.empty()) {
      const int pc = wl.back();
      wl.pop_back();
      for (int t : pred[pc]) {
        const int d = bw[pc] == kMany ? kMany : bw[pc] + weight(t);
        if (bw[t] == kUnset) bw[t] = d;
        else if (bw[t] != d && bw[t] != kMany) bw[t] = kMany;
        else continue;
        wl.push_back(t);
      }
    }
  }
  // group length: runes from `open` to `close` on every path between them
  int glen = kUnset;
  {
    std::vector<int> d(n, kUnset);
    std::vector<int> wl{open};
    d[open] = 0;
    while (!wl.empty()) {
      const int pc = wl.back();
      wl.pop_back();
      if (pc == close) continue;
      int o[2];
      const int k = succ(pc, o);
      for (int q = 0; q < k; ++q) {
        const int t = o[q];
        if (t <= 0 || t >= n) continue;
        const int nd = d[pc] == kMany ? kMany : d[pc] + weight(pc);
        if (d[t] == kUnset) d[t] = nd;
        else if (d[t] != nd && d[t] != kMany) d[t] = kMany;
        else continue;
        wl.push_back(t);
      }
    }
    glen = d[close];
  }
  // a CAP on a cycle would show up as "many" below only if the cycle consumes;
  // an empty cycle through it is rejected outright
  auto on_cycle = [&](int node) {
    std::vector<uint8_t> seen(n, 0);
    std::vector<int> st;
    int o[2];
    for (int k = succ(node, o); k-- > 0;) st.push_back(o[k]);
    while (!st.empty()) {
      const int pc = st.back();
      st.pop_back();
      if (pc <= 0 || pc >= n || seen[pc]) continue;
      if (pc == node) return true;
      seen[pc] = 1;
      for (int k = succ(pc, o); k-- > 0;) st.push_back(o[k]);
    }
    return false;
  };
  if (on_cycle(open) || on_cycle(close)) return g;
  g.pre = fw[open] >= 0 ? fw[open] : -1;
  g.suf = bw[close] >= 0 ? bw[close] : -1;
  g.len = glen >= 0 ? glen : -1;
  g.valid = (g.pre >= 0 || (g.suf >= 0 && g.len >= 0)) && (g.suf >= 0 || (g.pre >= 0 && g.len >= 0));
  return g;
}

// Capture-group span by byte runs (see gre.h GroupRun).  With A the part of
// the program before the group's CAP pair, B the group and S the rest: on
// ASCII text, if no byte S can consume can be B's last byte, the match's
// trailing run of S-bytes is exactly S's text (the byte before it was consumed
// last by B); if no byte B can consume can be A's last byte, the run of
// B-bytes before that is exactly the group (the byte before it, if any, was
// consumed last by A).  Every parse of the match has these boundaries, so the
// leftmost-first one does too.  Sets are supersets from graph reachability.
GroupRun group_run(const Prog& p, uint32_t slot, int fixed_len) {
  GroupRun g;
  const int n = (int)p.inst.size();
  int open = -1, close = -1;
  for (int pc = 0; pc < n; ++pc) {
    const Inst& in = p.inst[pc];
    if (in.op != I_CAP) continue;
    if (in.arg == 2 * slot) {
      if (open >= 0) return g;
      open = pc;
    } else if (in.arg == 2 * slot + 1) {
      if (close >= 0) return g;
      close = pc;
    }
  }
  if (open < 0 || close < 0) return g;
  auto succ = [&](int pc, int* out) -> int {
    const Inst& in = p.inst[pc];
    switch (in.op) {
      case I_FAIL:
      case I_MATCH: return 0;
      case I_ALT: out[0] = (int)in.out; out[1] = (int)in.arg; return 2;
      default: out[0] = (int)in.out; return 1;
    }
  };
  auto consumes = [&](int pc) {
    const uint8_t op = p.inst[pc].op;
    return op == I_RUNE || op == I_RUNE1 || op == I_ANY || op == I_ANYNL;
  };
  auto bytes_of = [&](int pc, uint32_t* m) {  // ASCII bytes the instruction consumes
    const Inst& in = p.inst[pc];
    switch (in.op) {
      case I_RUNE:
        for (int k = 0; k < 4; ++k) m[k] |= p.classes[in.arg].ascii[k];
        break;
      case I_RUNE1:
        if (in.arg < 128) m[in.arg >> 5] |= 1u << (in.arg & 31);
        break;
      case I_ANY:
        for (int k = 0; k < 4; ++k) m[k] = ~0u;
        break;
      case I_ANYNL:
        for (int k = 0; k < 4; ++k) m[k] = ~0u;
        m['\n' >> 5] &= ~(1u << ('\n' & 31));
        break;
    }
  };
  // forward reachability from `from` (over every edge), never entering `stop`
  auto reach = [&](int from, int stop) {
    std::vector<uint8_t> seen(n, 0);
    std::vector<int> st{from};
    while (!st.empty()) {
      const int pc = st.back();
      st.pop_back();
      if (pc <= 0 || pc >= n || pc == stop || seen[pc]) continue;
      seen[pc] = 1;
      int o[2];
      for (int k = succ(pc, o); k-- > 0;) st.push_back(o[k]);
    }
    return seen;
  };
  // the empty-width closure of `from` (no consuming instruction passed) meets `target`
  auto eps_reaches = [&](int from, int target) {
    std::vector<uint8_t> seen(n, 0);
    std::vector<int> st{from};
    while (!st.empty()) {
      const int pc = st.back();
      st.pop_back();
      if (pc <= 0 || pc >= n || seen[pc]) continue;
      if (pc == target) return true;
      seen[pc] = 1;
      if (consumes(pc) || p.inst[pc].op == I_MATCH) continue;
      int o[2];
      for (int k = succ(pc, o); k-- > 0;) st.push_back(o[k]);
    }
    return false;
  };
  // the group takes part in every match: MATCH unreachable around open / close
  {
    auto around = [&](int cut) {
      const std::vector<uint8_t> r = reach((int)p.start, cut);
      for (int pc = 1; pc < n; ++pc)
        if (r[pc] && p.inst[pc].op == I_MATCH) return true;
      return false;
    };
    if (around(open) || around(close)) return g;
  }
  if (eps_reaches((int)p.inst[open].out, close)) return g;  // the group may be empty
  const std::vector<uint8_t> from_start = reach((int)p.start, -1);
  const std::vector<uint8_t> in_group = reach((int)p.inst[open].out, close);  // B (and what loops back)
  const std::vector<uint8_t> after = reach((int)p.inst[close].out, -1);       // S
  uint32_t s_alpha[4] = {0, 0, 0, 0}, b_alpha[4] = {0, 0, 0, 0}, b_last[4] = {0, 0, 0, 0}, a_last[4] = {0, 0, 0, 0};
  for (int pc = 1; pc < n; ++pc) {
    if (!consumes(pc)) continue;
    if (after[pc]) bytes_of(pc, s_alpha);
    if (in_group[pc]) {
      bytes_of(pc, b_alpha);
      if (eps_reaches((int)p.inst[pc].out, close)) bytes_of(pc, b_last);
    }
    if (from_start[pc] && eps_reaches((int)p.inst[pc].out, open)) bytes_of(pc, a_last);
  }
  // (a group of fixed length starts len bytes before its end on ASCII text:
  // what A ends with does not matter then)
  for (int k = 0; k < 4; ++k)
    if ((s_alpha[k] & b_last[k]) || (fixed_len < 0 && (b_alpha[k] & a_last[k]))) return g;
  g.valid = true;
  g.len = fixed_len;
  for (int k = 0; k < 4; ++k) {
    g.s_alpha[k] = s_alpha[k];
    g.b_alpha[k] = b_alpha[k];
  }
  return g;
}

// Inst::vis rows: the start plus every instruction with >= 2 predecessors
// among the instructions reachable from the start.
static void assign_vis_rows(Prog* p) {
  const size_t n = p->inst.size();
  std::vector<uint32_t> indeg(n, 0);
  std::vector<uint8_t> seen(n, 0);
  std::vector<uint32_t> st{p->start};
  while (!st.empty()) {
    const uint32_t pc = st.back();
    st.pop_back();
    if (pc == 0 || pc >= n || seen[pc]) continue;
    seen[pc] = 1;
    const Inst& in = p->inst[pc];
    if (in.op == I_FAIL || in.op == I_MATCH) continue;
    const uint32_t o[2] = {in.out, in.arg};
    for (int k = 0; k < (in.op == I_ALT ? 2 : 1); ++k)
      if (o[k] && o[k] < n) {
        ++indeg[o[k]];
        st.push_back(o[k]);
      }
  }
  p->nvis = 0;
  for (size_t pc = 0; pc < n; ++pc) {
    const bool row = seen[pc] && (pc == p->start || indeg[pc] >= 2);
    p->inst[pc].vis = row ? (uint16_t)p->nvis++ : kNoVis;
  }
}

bool compile(const std::string& pattern, Compiled* out, std::string* err) {
  try {
    Parser ps(pattern);
    Node* root = ps.parse();
    simplify(root);
    out->prog = Prog{};
    Compiler c(&out->prog);
    Frag f = c.compile(root);
    if (f.i == 0) {
      // pattern can never match: a program whose start is FAIL
      out->prog.start = 0;
      out->prog.inst.push_back(Inst{I_MATCH, 0, 0, 0, 0});
    } else {
      c.finish(f);
    }
    out->prog.ncap = 2 * (ps.ncap() + 1);
    out->prog.cap_names = ps.names();
    assign_vis_rows(&out->prog);
    if (out->prog.inst.size() >= 65535) {
      *err = "expression too large";
      return false;
    }
    A a = analyze(root);
    out->anchor = a.best;
    out->can_match_empty = a.nullable;
    out->min_len = a.minlen;
    out->max_len = a.maxlen;
    if (out->anchor.valid && a.nullable) out->anchor.valid = false;  // defensive
    out->literal_exact = false;
    if (out->anchor.valid && a.exact && !has_assert(root) && out->anchor.off_min == 0 && out->anchor.off_max == 0 &&
        out->anchor.lits.size() == a.ex.size()) {
      bool same = true;
      for (auto& l : a.ex) same &= std::find(out->anchor.lits.begin(), out->anchor.lits.end(), l) != out->anchor.lits.end();
      out->literal_exact = same;
    }
    return true;
  } catch (const SyntaxError& e) {
    *err = "error parsing regexp: " + e.msg;
    return false;
  }
}

}  // namespace gre
