// findings.cpp — host finishing of kept locations into SecretFindings.
//
// Restates, on the caller's host copy of the content, the tail of
// Scanner.Scan: censorLocation over every kept location (scanner.go:425-429,
// 454-462), toFinding/findLocation against the FINAL censored buffer
// (scanner.go:433-435, 464-537) and the (RuleID, Match) sort (scanner.go:441-446).
// Line numbers come from the device (k_lines); the Code window is cut by
// walking at most a few lines around the location instead of splitting the
// whole file per finding.
#include <algorithm>
#include <cstring>

#include "engine.h"

namespace tsg {

namespace {

// Byte offset of the start of 0-based line `target`, scanning back from a
// position inside line `cur` (cur >= target).
// start of the line holding byte pos-1's successor: one past the last '\n' before pos
size_t line_begin(const uint8_t* c, size_t pos) {
  const void* q = pos ? memrchr(c, '\n', pos) : nullptr;
  return q ? (size_t)((const uint8_t*)q - c) + 1 : 0;
}

size_t line_start_back(const uint8_t* c, size_t pos, uint32_t cur, uint32_t target) {
  size_t p = line_begin(c, pos);  // the start of line `cur`
  while (cur > target && p > 0) {
    // p is the start of line cur; previous line ends at p-1 ('\n')
    p = line_begin(c, p - 1);
    --cur;
  }
  return p;
}

}  // namespace

bool build_findings(ResultImpl* R, const tsg_ruleset* rs, const tsg_file* files, size_t n_files) {
  R->findings.assign(n_files, {});
  R->lines.clear();
  R->strs.clear();
  // group locations per file, in Scan's (rule, position) order
  std::vector<std::vector<const tsg_loc*>> per(n_files);
  for (auto& L : R->locs) per[L.file].push_back(&L);
  for (size_t f = 0; f < n_files; ++f) {
    auto& v = per[f];
    if (v.empty()) continue;
    std::sort(v.begin(), v.end(), [](const tsg_loc* a, const tsg_loc* b) {
      if (a->rule != b->rule) return a->rule < b->rule;
      if (a->start != b->start) return a->start < b->start;
      return a->end < b->end;
    });
    const uint8_t* src = files[f].data;
    const size_t n = files[f].len;
    std::string censored(reinterpret_cast<const char*>(src), n);
    for (auto* L : v) {
      if (L->end > n || L->start > L->end) return false;
      memset(&censored[L->start], '*', L->end - L->start);
    }
    const uint8_t* c = reinterpret_cast<const uint8_t*>(censored.data());
    uint32_t total_lines = 1;  // len(bytes.Split(content, "\n"))
    for (const uint8_t* q = c; (q = (const uint8_t*)memchr(q, '\n', n - (q - c))) != nullptr; ++q) ++total_lines;
    std::vector<tsg_finding> out;
    for (auto* L : v) {
      const size_t start = L->start, end = L->end;
      // match window (scanner.go:484-502)
      size_t ls = line_begin(c, start);
      const void* nl = start < n ? memchr(c + start, '\n', n - start) : nullptr;
      size_t le = nl ? (size_t)((const uint8_t*)nl - c) : n;
      if (le - ls > 100) {
        ls = start >= 30 ? start - 30 : 0;
        le = end + 20 > n ? n : end + 20;
      }
      R->strs.emplace_back(censored.substr(ls, le - ls));
      const std::string& match = R->strs.back();
      // code lines (scanner.go:505-534), 0-based line numbers
      const uint32_t sl = L->start_line - 1, el = L->end_line - 1;
      const uint32_t cs = sl >= 2 ? sl - 2 : 0;
      const uint32_t ce = std::min<uint32_t>(el + 2, total_lines);
      R->lines.emplace_back();
      auto& lines = R->lines.back();
      size_t p = line_start_back(c, start, sl, cs);
      bool found_first = false;
      for (uint32_t ln = cs; ln < ce && p <= n; ++ln) {
        const void* nq = p < n ? memchr(c + p, '\n', n - p) : nullptr;
        size_t q = nq ? (size_t)((const uint8_t*)nq - c) : n;
        R->strs.emplace_back(censored.substr(p, q - p));
        const std::string& txt = R->strs.back();
        const bool cause = ln >= sl && ln <= el;
        tsg_line tl{};
        tl.number = ln + 1;
        tl.content = txt.data();
        tl.content_len = txt.size();
        tl.is_cause = cause;
        tl.first_cause = !found_first && cause;
        tl.last_cause = 0;
        found_first = found_first || cause;
        lines.push_back(tl);
        p = q + 1;
      }
      for (size_t k = lines.size(); k-- > 0;) {
        if (lines[k].is_cause) {
          lines[k].last_cause = 1;
          break;
        }
      }
      tsg_finding fd{};
      fd.file = (uint32_t)f;
      fd.rule = L->rule;
      fd.start_line = L->start_line;
      fd.end_line = L->end_line;
      fd.match = match.data();
      fd.match_len = match.size();
      fd.lines = lines.data();
      fd.n_lines = lines.size();
      fd.start = start;
      fd.end = end;
      out.push_back(fd);
    }
    std::stable_sort(out.begin(), out.end(), [&](const tsg_finding& a, const tsg_finding& b) {
      const std::string& ia = rs->rules[a.rule].id;
      const std::string& ib = rs->rules[b.rule].id;
      if (ia != ib) return ia < ib;
      return std::string(a.match, a.match_len) < std::string(b.match, b.match_len);
    });
    R->findings[f] = std::move(out);
  }
  R->have_findings = true;
  return true;
}

}  // namespace tsg
