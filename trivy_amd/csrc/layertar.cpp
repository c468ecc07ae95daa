// layertar.cpp — container-image layer walker feeding the batched analyzer.
//
// Restates walker.LayerTar.Walk (pkg/fanal/walker/tar.go:35-103) over a layer
// tar that is already in host memory (read or mmap'd by the caller): opaque
// directory markers (.wh..wh..opq, tar.go:51-54), whiteouts (.wh.<name>,
// tar.go:56-61), SkipDirs/SkipFiles by doublestar glob (walk.go:39-53),
// descendants of skipped directories (underSkippedDir, tar.go:106-117), and
// every remaining directory/regular entry in archive order.  Nothing is
// copied: an entry's content is a (offset, size) span of the caller's tar, so
// a whole layer goes to tsg_analyze (which packs pinned staging with threads
// and overlaps the H2D) in one call instead of one cgo call per file
// (SURVEY.md §8f rank 2).
//
// Header decoding follows Go's archive/tar Reader (go1.22): USTAR prefix
// joined to the name, GNU 'L'/'K' long names, PAX 'x' records (path, size),
// TypeRegA ('\0') read as TypeReg, or TypeDir for a name ending in '/',
// octal or base-256 numeric fields, header checksum (unsigned or signed sum),
// and end of archive at a zero block.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <system_error>
#include <thread>
#include <vector>

#include "engine.h"

namespace tsg {
void set_last_error(const std::string& m);
bool host_allow_path(const tsg_ruleset* rs, const uint8_t* path, size_t len);
}

struct tsg_tar_walk {
  std::vector<tsg_tar_entry> entries;
  std::vector<std::string> paths;  // backing store of entries[i].path
  std::vector<std::string> opq_dirs, wh_files;
};

namespace {

constexpr size_t kBlock = 512;

// path.Clean (Go, lexical).
// True when path.Clean would return p unchanged (the common case in layers):
// no empty, "." or ".." element and no trailing '/'.
bool already_clean(const std::string& p) {
  if (p.empty() || p.back() == '/') return p == "/";
  size_t i = p[0] == '/' ? 1 : 0;
  while (i < p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    size_t n = j - i;
    if (n == 0 || (n == 1 && p[i] == '.') || (n == 2 && p[i] == '.' && p[i + 1] == '.')) return false;
    i = j + 1;
  }
  return true;
}

std::string go_path_clean(const std::string& p) {
  if (already_clean(p)) return p;
  if (p.empty()) return ".";
  bool rooted = p[0] == '/';
  std::vector<std::string> parts;
  size_t i = 0, n = p.size();
  while (i < n) {
    while (i < n && p[i] == '/') i++;
    size_t j = i;
    while (j < n && p[j] != '/') j++;
    std::string e = p.substr(i, j - i);
    i = j;
    if (e.empty() || e == ".") continue;
    if (e == "..") {
      if (!parts.empty() && parts.back() != "..")
        parts.pop_back();
      else if (!rooted)
        parts.push_back("..");
      continue;
    }
    parts.push_back(e);
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < parts.size(); k++) {
    if (k) out += '/';
    out += parts[k];
  }
  if (out.empty()) return ".";
  return out;
}

std::string trim_left_slash(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && s[i] == '/') i++;
  return s.substr(i);
}

// path.Join(dir, name) for the whiteout target.
std::string go_path_join(const std::string& a, const std::string& b) {
  if (a.empty() && b.empty()) return "";
  if (a.empty()) return go_path_clean(b);
  if (b.empty()) return go_path_clean(a);
  return go_path_clean(a + "/" + b);
}

// ---- doublestar.Match (github.com/bmatcuk/doublestar/v4) -------------------
// '*' any run of non-'/' bytes, '?' one non-'/' byte, '[...]' a class ('!' or
// '^' negates, ranges, '\' escapes), '{a,b}' alternatives, '**' as a whole
// path component zero or more components; '\' escapes the next byte.
bool glob_seg(const std::string& pat, size_t pi, const std::string& s, size_t si);

// Expand the first top-level {..} alternative group; returns false if none.
bool expand_braces(const std::string& pat, std::vector<std::string>* out) {
  size_t open = std::string::npos;
  int depth = 0;
  std::vector<size_t> commas;
  for (size_t i = 0; i < pat.size(); i++) {
    char c = pat[i];
    if (c == '\\') {
      i++;
      continue;
    }
    if (c == '[') {  // skip a class
      size_t j = i + 1;
      if (j < pat.size() && (pat[j] == '!' || pat[j] == '^')) j++;
      if (j < pat.size() && pat[j] == ']') j++;
      while (j < pat.size() && pat[j] != ']') j += pat[j] == '\\' ? 2 : 1;
      i = j;
      continue;
    }
    if (c == '{') {
      if (depth == 0) open = i, commas.clear();
      depth++;
    } else if (c == ',' && depth == 1) {
      commas.push_back(i);
    } else if (c == '}' && depth > 0) {
      if (--depth == 0) {
        std::string pre = pat.substr(0, open), post = pat.substr(i + 1);
        size_t a = open + 1;
        commas.push_back(i);
        for (size_t cpos : commas) {
          out->push_back(pre + pat.substr(a, cpos - a) + post);
          a = cpos + 1;
        }
        return true;
      }
    }
  }
  return false;
}

bool class_match(const std::string& pat, size_t* pi, unsigned char ch, bool* ok) {
  size_t i = *pi + 1;
  bool neg = false;
  if (i < pat.size() && (pat[i] == '!' || pat[i] == '^')) neg = true, i++;
  bool hit = false, first = true;
  while (i < pat.size() && (first || pat[i] != ']')) {
    first = false;
    unsigned char lo = pat[i];
    if (lo == '\\' && i + 1 < pat.size()) lo = pat[++i];
    i++;
    unsigned char hi = lo;
    if (i + 1 < pat.size() && pat[i] == '-' && pat[i + 1] != ']') {
      hi = pat[i + 1];
      if (hi == '\\' && i + 2 < pat.size()) hi = pat[++i + 1];
      i += 2;
    }
    if (lo <= ch && ch <= hi) hit = true;
  }
  if (i >= pat.size()) {  // unterminated class: bad pattern
    *ok = false;
    return false;
  }
  *pi = i + 1;
  return hit != neg;
}

thread_local bool g_bad_pattern = false;

bool glob_seg(const std::string& pat, size_t pi, const std::string& s, size_t si) {
  while (pi < pat.size()) {
    char c = pat[pi];
    if (c == '*') {
      bool dstar = pi + 1 < pat.size() && pat[pi + 1] == '*' && (pi == 0 || pat[pi - 1] == '/') &&
                   (pi + 2 == pat.size() || pat[pi + 2] == '/');
      if (dstar) {
        if (pi + 2 == pat.size()) return true;  // "**" at the end: everything below
        // "**/rest": rest against si and after every '/' from si on
        size_t rest = pi + 3;
        if (glob_seg(pat, rest, s, si)) return true;
        for (size_t k = si; k < s.size(); k++)
          if (s[k] == '/' && glob_seg(pat, rest, s, k + 1)) return true;
        return false;
      }
      while (pi < pat.size() && pat[pi] == '*') pi++;
      for (size_t k = si;; k++) {
        if (glob_seg(pat, pi, s, k)) return true;
        if (k >= s.size() || s[k] == '/') return false;
      }
    }
    if (si >= s.size()) {
      // "a/**" also matches "a": a trailing "/**" may match nothing
      return pat.compare(pi, std::string::npos, "/**") == 0;
    }
    if (c == '?') {
      if (s[si] == '/') return false;
      pi++, si++;
      continue;
    }
    if (c == '[') {
      bool ok = true;
      if (s[si] == '/') return false;
      bool m = class_match(pat, &pi, (unsigned char)s[si], &ok);
      if (!ok) {
        g_bad_pattern = true;
        return false;
      }
      if (!m) return false;
      si++;
      continue;
    }
    if (c == '\\' && pi + 1 < pat.size()) pi++, c = pat[pi];
    if (s[si] != c) return false;
    pi++, si++;
  }
  return si == s.size();
}

bool doublestar_match(const std::string& pat, const std::string& s, bool* bad) {
  std::vector<std::string> alts;
  if (expand_braces(pat, &alts)) {
    for (auto& a : alts) {
      if (doublestar_match(a, s, bad)) return true;
      if (*bad) return false;
    }
    return false;
  }
  g_bad_pattern = false;
  bool m = glob_seg(pat, 0, s, 0);
  *bad = g_bad_pattern;
  return m && !*bad;
}

// walker.SkipPath (walk.go:39-53): a bad pattern ends the search (false).
bool skip_path(const std::string& path, const std::vector<std::string>& pats) {
  if (pats.empty()) return false;
  std::string p = trim_left_slash(path);
  for (auto& pat : pats) {
    bool bad = false;
    bool m = doublestar_match(pat, p, &bad);
    if (bad) return false;
    if (m) return true;
  }
  return false;
}

std::vector<std::string> split_clean(const std::string& p) {
  std::vector<std::string> v;
  if (p == ".") return v;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    v.push_back(p.substr(i, j - i));
    i = j + 1;
  }
  return v;
}

// underSkippedDir (tar.go:106-117): filepath.Rel(skipDir, filePath) does not
// start with "../".  Both paths are clean and relative, so Rel is lexical:
// ".." per unshared base component, then the target's remaining components.
bool under_skipped_dir(const std::string& file, const std::vector<std::string>& dirs) {
  if (dirs.empty()) return false;
  auto t = split_clean(file);
  for (auto& d : dirs) {
    auto b = split_clean(go_path_clean(d));
    size_t c = 0;
    while (c < b.size() && c < t.size() && b[c] == t[c]) c++;
    size_t ups = b.size() - c, rest = t.size() - c;
    // Rel = "../"*ups + rest: "" -> ".", ".." alone does not start with "../"
    if (ups == 0 || (ups == 1 && rest == 0)) return true;
  }
  return false;
}

std::vector<std::string> clean_skip_paths(const char* const* v, size_t n) {
  std::vector<std::string> out;
  for (size_t i = 0; i < n; i++) out.push_back(trim_left_slash(go_path_clean(v[i] ? v[i] : "")));
  return out;
}

std::string cstr_field(const uint8_t* p, size_t n) {
  size_t k = 0;
  while (k < n && p[k]) k++;
  return std::string((const char*)p, k);
}

bool parse_numeric(const uint8_t* p, size_t n, int64_t* out) {
  if (n && (p[0] & 0x80)) {  // base-256 (GNU)
    uint64_t v = p[0] & 0x7f;
    if (p[0] & 0x40) return false;  // negative
    for (size_t i = 1; i < n; i++) {
      if (v >> 56) return false;
      v = (v << 8) | p[i];
    }
    *out = (int64_t)v;
    return true;
  }
  size_t i = 0;
  while (i < n && (p[i] == ' ' || p[i] == 0)) i++;
  int64_t v = 0;
  bool any = false;
  for (; i < n && p[i] >= '0' && p[i] <= '7'; i++) v = v * 8 + (p[i] - '0'), any = true;
  for (; i < n; i++)
    if (p[i] != ' ' && p[i] != 0) return false;
  *out = any ? v : 0;
  return true;
}

bool checksum_ok(const uint8_t* h) {
  int64_t want;
  if (!parse_numeric(h + 148, 8, &want)) return false;
  // sums over the block with the checksum field read as spaces; plain loops
  // the compiler vectorises (this runs once per member)
  uint32_t u = 0;
  int32_t s = 0;
  for (size_t i = 0; i < kBlock; i++) u += h[i];
  for (size_t i = 0; i < kBlock; i++) s += (int8_t)h[i];
  for (size_t i = 148; i < 156; i++) {
    u += ' ' - h[i];
    s += ' ' - (int8_t)h[i];
  }
  return want == (int64_t)u || want == (int64_t)s;
}

bool zero_block(const uint8_t* h) {
  uint64_t acc = 0;
  for (size_t i = 0; i < kBlock; i += 8) {
    uint64_t v;
    memcpy(&v, h + i, 8);
    acc |= v;
  }
  return acc == 0;
}

// PAX records "%d key=value\n" (archive/tar parsePAX).
bool parse_pax(const uint8_t* p, size_t n, std::string* path, int64_t* size, bool* has_path, bool* has_size) {
  size_t i = 0;
  while (i < n) {
    size_t sp = i;
    while (sp < n && p[sp] != ' ') sp++;
    if (sp >= n) return false;
    size_t len = 0;
    for (size_t k = i; k < sp; k++) {
      if (p[k] < '0' || p[k] > '9') return false;
      len = len * 10 + (p[k] - '0');
    }
    if (len == 0 || i + len > n || p[i + len - 1] != '\n') return false;
    std::string rec((const char*)p + sp + 1, i + len - 1 - (sp + 1));
    size_t eq = rec.find('=');
    if (eq == std::string::npos) return false;
    std::string key = rec.substr(0, eq), val = rec.substr(eq + 1);
    if (key == "path") *path = val, *has_path = true;
    if (key == "size") {
      char* e = nullptr;
      long long v = strtoll(val.c_str(), &e, 10);
      if (!e || *e || v < 0) return false;
      *size = v, *has_size = true;
    }
    i += len;
  }
  return true;
}

int fail(const std::string& m) {
  tsg::set_last_error(m);
  return -1;
}

}  // namespace

extern "C" {

int tsg_layer_tar_walk(const uint8_t* tar, size_t len, const char* const* skip_files, size_t n_skip_files,
                       const char* const* skip_dirs, size_t n_skip_dirs, tsg_tar_walk** out) {
  if (!out) return fail("tsg_layer_tar_walk: null out");
  *out = nullptr;
  if (!tar && len) return fail("tsg_layer_tar_walk: null tar with nonzero length");
  try {
    auto* w = new tsg_tar_walk();
    auto sf = clean_skip_paths(skip_files, n_skip_files), sd = clean_skip_paths(skip_dirs, n_skip_dirs);
    std::vector<std::string> skipped_dirs;
    std::string long_name, pax_path;
    int64_t pax_size = -1;
    bool have_long = false, have_pax_path = false;
    size_t off = 0;
    auto err = [&](const std::string& m) {
      delete w;
      return fail("failed to extract the archive: " + m);
    };
    while (true) {
      if (off + kBlock > len) {
        if (off == len) break;  // io.EOF at a block boundary
        return err("unexpected EOF");
      }
      const uint8_t* h = tar + off;
      if (zero_block(h)) {
        // archive/tar readHeader: a zero block must be followed by EOF or a
        // second zero block; a zero block then a header is ErrHeader
        const size_t nx = off + kBlock;
        if (nx == len) break;                                  // io.EOF after one block
        if (nx + kBlock > len) return err("unexpected EOF");   // partial second block
        if (zero_block(tar + nx)) break;                       // normal end of archive
        return err("archive/tar: invalid tar header");
      }
      if (!checksum_ok(h)) return err("archive/tar: invalid tar header");
      int64_t size;
      if (!parse_numeric(h + 124, 12, &size) || size < 0) return err("archive/tar: invalid tar header");
      char type = (char)h[156];
      bool ustar = memcmp(h + 257, "ustar\0", 6) == 0;
      size_t data = off + kBlock;
      if (type == 'x' || type == 'L' || type == 'K' || type == 'g') {
        if ((uint64_t)size > len - data) return err("unexpected EOF");
      }
      size_t next = data + (((uint64_t)size + kBlock - 1) / kBlock) * kBlock;
      if (type == 'x') {  // PAX header for the next entry
        bool hp = false, hs = false;
        std::string pp;
        int64_t ps = -1;
        if (!parse_pax(tar + data, size, &pp, &ps, &hp, &hs)) return err("archive/tar: invalid tar header");
        if (hp) pax_path = pp, have_pax_path = true;
        if (hs) pax_size = ps;
        off = next;
        continue;
      }
      if (type == 'L' || type == 'K') {  // GNU long name / long link name
        if (type == 'L') long_name = cstr_field(tar + data, size), have_long = true;
        off = next;
        continue;
      }
      std::string name = cstr_field(h, 100);
      if (ustar) {
        std::string prefix = cstr_field(h + 345, 155);
        if (!prefix.empty()) name = prefix + "/" + name;
      }
      if (have_long) name = long_name;
      if (have_pax_path) name = pax_path;
      if (pax_size >= 0) {
        size = pax_size;
        next = data + (((uint64_t)size + kBlock - 1) / kBlock) * kBlock;
      }
      have_long = have_pax_path = false;
      pax_size = -1;
      if (type == '\0') type = (!name.empty() && name.back() == '/') ? '5' : '0';
      bool has_data = !(type == '1' || type == '2' || type == '3' || type == '4' || type == '5' || type == '6');
      if (has_data && (uint64_t)size > len - data) return err("unexpected EOF");
      off = has_data ? next : data;
      if (off + kBlock <= len)  // the next header is a cache/TLB miss: start it before this entry's string work
        for (size_t l = 0; l < kBlock; l += 64) __builtin_prefetch(tar + off + l);

      // tar.go:47-49: path.Clean, then strip leading '/'
      std::string fp = trim_left_slash(go_path_clean(name));
      size_t slash = fp.rfind('/');
      std::string dir = slash == std::string::npos ? "" : fp.substr(0, slash + 1);
      std::string base = slash == std::string::npos ? fp : fp.substr(slash + 1);
      if (base == ".wh..wh..opq") {  // tar.go:51-54
        w->opq_dirs.push_back(dir);
        continue;
      }
      if (base.compare(0, 4, ".wh.") == 0) {  // tar.go:56-61
        w->wh_files.push_back(go_path_join(dir, base.substr(4)));
        continue;
      }
      if (type == '5') {
        if (skip_path(fp, sd)) {
          skipped_dirs.push_back(fp);
          continue;
        }
      } else if (type == '0') {  // TypeCont '7' falls to default, as in Go
        if (skip_path(fp, sf)) continue;
      } else {
        continue;  // links, devices, fifos, global PAX: no content (tar.go:75-77)
      }
      if (under_skipped_dir(fp, skipped_dirs)) continue;
      int64_t mode = 0;
      parse_numeric(h + 100, 8, &mode);
      tsg_tar_entry e{};
      e.offset = type == '5' ? 0 : data;
      e.size = type == '5' ? 0 : (uint64_t)size;
      e.mode = (uint32_t)mode;
      e.is_dir = type == '5';
      w->paths.push_back(fp);
      w->entries.push_back(e);
    }
    for (size_t i = 0; i < w->entries.size(); i++) {
      w->entries[i].path = w->paths[i].c_str();
      w->entries[i].path_len = w->paths[i].size();
    }
    *out = w;
    return 0;
  } catch (const std::exception& ex) {
    return fail(std::string("internal error: ") + ex.what());
  }
}

size_t tsg_tar_walk_entry_count(const tsg_tar_walk* w) { return w ? w->entries.size() : 0; }
const tsg_tar_entry* tsg_tar_walk_entries(const tsg_tar_walk* w) {
  return w && !w->entries.empty() ? w->entries.data() : nullptr;
}
size_t tsg_tar_walk_opq_count(const tsg_tar_walk* w) { return w ? w->opq_dirs.size() : 0; }
const char* tsg_tar_walk_opq_dir(const tsg_tar_walk* w, size_t i) {
  return w && i < w->opq_dirs.size() ? w->opq_dirs[i].c_str() : nullptr;
}
size_t tsg_tar_walk_wh_count(const tsg_tar_walk* w) { return w ? w->wh_files.size() : 0; }
const char* tsg_tar_walk_wh_file(const tsg_tar_walk* w, size_t i) {
  return w && i < w->wh_files.size() ? w->wh_files[i].c_str() : nullptr;
}
void tsg_tar_walk_free(tsg_tar_walk* w) { delete w; }

// SecretAnalyzer.Required (pkg/fanal/analyzer/secret/secret.go:115-153).
static bool secret_required(const tsg_ruleset* rs, const std::string& fp, uint64_t size,
                            const std::string& config_base) {
  static const char* kSkipFiles[] = {"go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml",
                                     "Pipfile.lock", "Gemfile.lock"};  // secret.go:28-36
  static const char* kSkipExts[] = {".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket",
                                    ".deb", ".rpm", ".zip", ".gz", ".gzip", ".tar", ".pyc"};  // :38-41
  if (size < 10) return false;
  const std::string_view v(fp);  // (views: no allocation per file)
  const size_t slash = v.rfind('/');
  const std::string_view dir = slash == std::string_view::npos ? std::string_view() : v.substr(0, slash + 1);
  const std::string_view name = slash == std::string_view::npos ? v : v.substr(slash + 1);
  for (size_t i = 0; i <= dir.size();) {  // strings.Split(dir, "/") contains .git / node_modules
    size_t j = dir.find('/', i);
    if (j == std::string_view::npos) j = dir.size();
    const std::string_view c = dir.substr(i, j - i);
    if (c == ".git" || c == "node_modules") return false;
    i = j + 1;
  }
  for (const char* f : kSkipFiles)
    if (name == f) return false;
  if (config_base == fp) return false;
  const size_t dot = name.rfind('.');
  const std::string_view ext = dot == std::string_view::npos ? std::string_view() : name.substr(dot);  // filepath.Ext
  for (const char* x : kSkipExts)
    if (ext == x) return false;
  return !tsg::host_allow_path(rs, (const uint8_t*)fp.data(), fp.size());
}

// filepath.Base (Go): "" -> ".", trailing slashes dropped, "/" -> "/".
static std::string go_base(const char* p) {
  std::string s = p ? p : "";
  if (s.empty()) return ".";
  while (s.size() > 1 && s.back() == '/') s.pop_back();
  if (s == "/") return "/";
  size_t k = s.rfind('/');
  return k == std::string::npos ? s : s.substr(k + 1);
}

int tsg_analyze_layer(tsg_engine* e, const tsg_ruleset* rs, const uint8_t* tar, size_t len,
                      const tsg_tar_walk* w, const char* config_path, uint32_t* kept, size_t* n_kept,
                      tsg_result** out) {
  if (!rs || !w || !n_kept || !out || (!tar && len)) return fail("tsg_analyze_layer: null argument");
  try {
    std::string cb = go_base(config_path);
    std::vector<tsg_file> files;
    std::vector<std::string> paths;
    std::vector<uint32_t> idx;
    // Required per regular file, in parallel (the global allow-path regexes
    // run on the host Pike VM; ~µs per path), then kept in walk order.
    size_t ne = w->entries.size();
    std::vector<uint8_t> req(ne, 0);
    for (size_t i = 0; i < ne; i++)
      if (!w->entries[i].is_dir && w->entries[i].offset + w->entries[i].size > len)
        return fail("tsg_analyze_layer: walk does not belong to this tar");
    auto work = [&](size_t a, size_t b) {
      for (size_t i = a; i < b; i++) {
        const tsg_tar_entry& en = w->entries[i];
        // directories: AnalyzerGroup.AnalyzeFile (analyzer.go:398-400)
        req[i] = !en.is_dir && secret_required(rs, w->paths[i], en.size, cb);
      }
    };
    size_t nt = std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()), ne / 4096 + 1});
    if (nt <= 1) {
      work(0, ne);
    } else {
      // a thread that cannot be started leaves its range to this thread; the
      // started ones are always joined (no std::terminate on unwinding)
      std::vector<std::thread> ts;
      size_t per = (ne + nt - 1) / nt;
      size_t done_to = 0;
      for (size_t t = 0; t < nt; t++) {
        try {
          ts.emplace_back(work, std::min(ne, t * per), std::min(ne, (t + 1) * per));
          done_to = std::min(ne, (t + 1) * per);
        } catch (const std::system_error&) {
          break;
        }
      }
      if (done_to < ne) work(done_to, ne);
      for (auto& t : ts) t.join();
    }
    for (size_t i = 0; i < ne; i++) {
      if (!req[i]) continue;
      paths.push_back("/" + w->paths[i]);  // Dir == "" (image.go:269) -> secret.go:95-98
      idx.push_back((uint32_t)i);
    }
    files.resize(idx.size());
    for (size_t k = 0; k < idx.size(); k++) {
      const tsg_tar_entry& en = w->entries[idx[k]];
      files[k].data = tar + en.offset;
      files[k].len = en.size;
      files[k].path = paths[k].c_str();
    }
    if (kept) memcpy(kept, idx.data(), idx.size() * sizeof(uint32_t));
    *n_kept = idx.size();
    return tsg_analyze(e, rs, files.data(), files.size(), out);
  } catch (const std::exception& ex) {
    return fail(std::string("internal error: ") + ex.what());
  }
}

int tsg_glob_match(const char* pattern, const char* path, int* matched) {
  if (!pattern || !path || !matched) return fail("tsg_glob_match: null argument");
  bool bad = false;
  *matched = doublestar_match(pattern, path, &bad) ? 1 : 0;
  return bad ? fail("syntax error in pattern") : 0;
}

}  // extern "C"
