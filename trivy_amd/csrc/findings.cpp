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
#include <string>
#include <utility>
#include <vector>

#include "engine.h"

namespace tsg {

namespace {

// The FINAL censored buffer of scanner.go:425-429 without materialising it:
// the caller's bytes plus the union of the kept locations, read as '*'.
// Newline searches skip censored bytes, so lines are those of the censored
// buffer (a censored multi-line match joins its lines, as in Go).
struct CensoredView {
  const uint8_t* o;
  size_t n;
  std::vector<std::pair<size_t, size_t>> iv;  // sorted, disjoint [a, b)

  CensoredView(const uint8_t* data, size_t len, const std::vector<const tsg_loc*>& locs) : o(data), n(len) {
    for (auto* L : locs)
      if (L->end > L->start) iv.push_back({(size_t)L->start, (size_t)L->end});
    std::sort(iv.begin(), iv.end());
    size_t k = 0;
    for (auto& r : iv) {
      if (k && r.first <= iv[k - 1].second) iv[k - 1].second = std::max(iv[k - 1].second, r.second);
      else iv[k++] = r;
    }
    iv.resize(k);
  }
  // the interval holding byte i, or nullptr
  const std::pair<size_t, size_t>* holder(size_t i) const {
    auto it = std::upper_bound(iv.begin(), iv.end(), std::make_pair(i, (size_t)-1));
    if (it == iv.begin()) return nullptr;
    --it;
    return i < it->second ? &*it : nullptr;
  }
  // first '\n' at or after `from` (n if none)
  size_t next_nl(size_t from) const {
    while (from < n) {
      const void* q = memchr(o + from, '\n', n - from);
      if (!q) return n;
      const size_t i = (size_t)((const uint8_t*)q - o);
      const auto* h = holder(i);
      if (!h) return i;
      from = h->second;
    }
    return n;
  }
  // start of the line holding position pos: one past the last '\n' before pos
  size_t line_begin(size_t pos) const {
    while (pos) {
      const void* q = memrchr(o, '\n', pos);
      if (!q) return 0;
      const size_t i = (size_t)((const uint8_t*)q - o);
      const auto* h = holder(i);
      if (!h) return i + 1;
      pos = h->first;
    }
    return 0;
  }
  std::string substr(size_t p, size_t q) const {
    std::string t(reinterpret_cast<const char*>(o) + p, q - p);
    auto it = std::upper_bound(iv.begin(), iv.end(), std::make_pair(p, (size_t)-1));
    if (it != iv.begin()) --it;
    for (; it != iv.end() && it->first < q; ++it) {
      const size_t a = std::max(it->first, p), b = std::min(it->second, q);
      if (a < b) memset(&t[a - p], '*', b - a);
    }
    return t;
  }
};

// Byte offset of the start of 0-based line `target`, scanning back from a
// position inside line `cur` (cur >= target).
size_t line_start_back(const CensoredView& c, size_t pos, uint32_t cur, uint32_t target) {
  size_t p = c.line_begin(pos);  // the start of line `cur`
  while (cur > target && p > 0) {
    p = c.line_begin(p - 1);  // previous line ends at p-1 ('\n')
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
    const size_t n = files[f].len;
    for (auto* L : v)
      if (L->end > n || L->start > L->end) return false;
    const CensoredView c(files[f].data, n, v);
    std::vector<tsg_finding> out;
    for (auto* L : v) {
      const size_t start = L->start, end = L->end;
      // match window (scanner.go:484-502)
      size_t ls = c.line_begin(start);
      size_t le = c.next_nl(start);
      if (le - ls > 100) {
        ls = start >= 30 ? start - 30 : 0;
        le = end + 20 > n ? n : end + 20;
      }
      R->strs.emplace_back(c.substr(ls, le));
      const std::string& match = R->strs.back();
      // code lines (scanner.go:505-534), 0-based line numbers; the window
      // ends at el + 2 or after the buffer's last line (p > n), whichever
      // comes first -- the min(.., len(lines)) of the reference
      const uint32_t sl = L->start_line - 1, el = L->end_line - 1;
      const uint32_t cs = sl >= 2 ? sl - 2 : 0;
      const uint32_t ce = el + 2;
      R->lines.emplace_back();
      auto& lines = R->lines.back();
      size_t p = line_start_back(c, start, sl, cs);
      bool found_first = false;
      for (uint32_t ln = cs; ln < ce && p <= n; ++ln) {
        const size_t q = c.next_nl(p);
        R->strs.emplace_back(c.substr(p, q));
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
