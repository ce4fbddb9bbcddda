// Native runtime for move2kube_amd: the CPU/file-system hot path.
//
// The reference (a Go binary) spends its planning time in (a) repeated
// filepath.Walk passes over the source tree (internal/common/utils.go:47-120,
// internal/source/dockerfile2kube.go:154-167), (b) running every file through
// buildkit's Dockerfile parser (dockerfile2kube.go:117-144) and (c) forking
// one /bin/sh per (detector x directory) pair serially
// (internal/containerizer/dockerfilecontainerizer.go:76-83).  This module
// provides native replacements:
//   walk()               one lexical-order lstat walk (Go filepath.Walk order)
//   sniff_dockerfiles()  multi-threaded "first non-ARG instruction" scan
//   run_commands()       bounded-parallel posix_spawn pool with captured stdout
//   proc_spawn/wait      one external tool without the subprocess module (proc_spawn.cpp)
//   procgroup_*          several tools waited for together in one poll loop (proc_spawn.cpp)
//   crc64_ecma/fnv64a    naming hashes (utils.go:292, compose/utils.go:121)
//   edit_distance_batch  weighted edit distance matrix (bit-parallel LCS for 1,1,2)
//   closest_batch        fused argmin over options for every query
// All long-running entry points release the GIL.

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <map>
#include <stdexcept>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <string>
#include <string_view>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <thread>
#include <time.h>
#include <tuple>
#include <unistd.h>
#include <vector>
#include <dirent.h>

extern char **environ;

namespace py = pybind11;

namespace {

// ----------------------------------------------------------------------------
// walk
// ----------------------------------------------------------------------------
enum Kind { K_FILE = 0, K_DIR = 1, K_SYMLINK = 2, K_OTHER = 3 };

struct WalkResult {
  std::vector<std::string> paths;
  std::vector<int> kinds;
  std::vector<std::pair<std::string, std::string>> errors;
};

// Go's syscall.Errno text: strerror with a lower-case first letter
// ("permission denied"), as filepath.Walk's errors print it.
static std::string go_errstr(int e) {
  std::string s = strerror(e);
  if (!s.empty() && s[0] >= 'A' && s[0] <= 'Z') s[0] = (char)(s[0] - 'A' + 'a');
  return s;
}

void walk_dir(const std::string &dir, WalkResult &r) {
  r.paths.push_back(dir);
  r.kinds.push_back(K_DIR);
  DIR *d = opendir(dir.c_str());
  if (!d) {
    r.errors.emplace_back(dir, std::string("open ") + dir + ": " + go_errstr(errno));
    return;
  }
  int dfd = dirfd(d);
  struct Ent {
    std::string name;
    unsigned char type;
  };
  std::vector<Ent> ents;
  while (struct dirent *e = readdir(d)) {
    if (e->d_name[0] == '.' && (e->d_name[1] == 0 || (e->d_name[1] == '.' && e->d_name[2] == 0)))
      continue;
    ents.push_back({e->d_name, e->d_type});
  }
  // Go sorts directory entries by name (byte order) before walking.
  std::sort(ents.begin(), ents.end(), [](const Ent &a, const Ent &b) { return a.name < b.name; });
  const std::string prefix = (dir == "/") ? std::string("/") : dir + "/";
  for (auto &e : ents) {
    std::string p = prefix + e.name;
    unsigned char t = e.type;
    if (t == DT_UNKNOWN) {
      struct stat st;
      if (fstatat(dfd, e.name.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0) {
        r.errors.emplace_back(p, std::string("lstat ") + p + ": " + go_errstr(errno));
        continue;
      }
      if (S_ISDIR(st.st_mode)) t = DT_DIR;
      else if (S_ISLNK(st.st_mode)) t = DT_LNK;
      else if (S_ISREG(st.st_mode)) t = DT_REG;
      else t = DT_FIFO;
    }
    if (t == DT_DIR) {
      walk_dir(p, r);
    } else {
      r.paths.push_back(p);
      r.kinds.push_back(t == DT_LNK ? K_SYMLINK : (t == DT_REG ? K_FILE : K_OTHER));
    }
  }
  closedir(d);
}

py::tuple walk(const std::string &root) {
  WalkResult r;
  {
    py::gil_scoped_release nogil;
    struct stat st;
    if (lstat(root.c_str(), &st) != 0) {
      r.errors.emplace_back(root, std::string("lstat ") + root + ": " + go_errstr(errno));
    } else if (S_ISDIR(st.st_mode)) {
      walk_dir(root, r);
    } else {
      r.paths.push_back(root);
      r.kinds.push_back(S_ISLNK(st.st_mode) ? K_SYMLINK : K_FILE);
    }
  }
  // File names are bytes: decode them like os.fsdecode (surrogateescape), so a
  // name that is not UTF-8 round-trips instead of failing the whole walk.
  auto fsdecode = [](const std::string &s) {
    PyObject *o = PyUnicode_DecodeFSDefaultAndSize(s.data(), static_cast<Py_ssize_t>(s.size()));
    if (!o) throw py::error_already_set();
    return py::reinterpret_steal<py::str>(o);
  };
  py::list paths(r.paths.size());
  for (size_t i = 0; i < r.paths.size(); i++) paths[i] = fsdecode(r.paths[i]);
  py::list errors(r.errors.size());
  for (size_t i = 0; i < r.errors.size(); i++)
    errors[i] = py::make_tuple(fsdecode(r.errors[i].first), fsdecode(r.errors[i].second));
  return py::make_tuple(paths, r.kinds, errors);
}

// ----------------------------------------------------------------------------
// Dockerfile sniffing (buildkit parser semantics for the first instructions)
// ----------------------------------------------------------------------------
// Returns, per file, the "Original" logical line of the first instruction that
// is not ARG if that instruction is FROM; "" otherwise.  A file that fails to
// parse (no instructions, over-long line, unreadable) yields "".

inline bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; }

std::string ltrim(const std::string &s) {
  size_t i = 0;
  while (i < s.size() && is_space((unsigned char)s[i])) i++;
  return s.substr(i);
}

// the instruction word of a logical line (buildkit splitCommand trims the line
// first: a line continued from an empty first line keeps its leading blanks)
std::string lower_word(const std::string &s) {
  size_t b = 0;
  while (b < s.size() && is_space((unsigned char)s[b])) b++;
  size_t i = b;
  while (i < s.size() && !is_space((unsigned char)s[i])) i++;
  std::string w = s.substr(b, i - b);
  for (auto &c : w) c = (char)tolower((unsigned char)c);
  return w;
}

// trim a trailing escape char followed by optional blanks: returns true if the line continues
bool trim_continuation(std::string &line, char esc) {
  size_t n = line.size();
  while (n > 0 && (line[n - 1] == ' ' || line[n - 1] == '\t')) n--;
  if (n > 0 && line[n - 1] == esc) {
    line.resize(n - 1);
    return true;
  }
  return false;
}

std::string sniff_one(const std::string &path) {
  const size_t kMaxLine = 64 * 1024;  // bufio.Scanner default token limit
  int fd = open(path.c_str(), O_RDONLY | O_NONBLOCK | O_CLOEXEC);  // a FIFO must not block: rejected by the S_ISREG check below
  if (fd < 0) return "";
  struct stat st;
  if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
    close(fd);
    return "";
  }
  std::string buf;
  size_t pos = 0;
  bool eof = false;
  auto fill = [&]() -> bool {
    if (eof) return false;
    char tmp[16384];
    ssize_t k = read(fd, tmp, sizeof(tmp));
    if (k <= 0) {
      eof = true;
      return false;
    }
    buf.append(tmp, (size_t)k);
    return true;
  };
  // read a physical line (without the newline); returns false at EOF with no data
  bool too_long = false;
  auto next_line = [&](std::string &out) -> bool {
    for (;;) {
      size_t nl = buf.find('\n', pos);
      if (nl != std::string::npos) {
        out.assign(buf, pos, nl - pos);
        pos = nl + 1;
        if (!out.empty() && out.back() == '\r') out.pop_back();
        if (out.size() > kMaxLine) too_long = true;
        return true;
      }
      if (buf.size() - pos > kMaxLine) {
        too_long = true;
        return false;
      }
      if (!fill()) {
        if (pos < buf.size()) {
          out.assign(buf, pos, buf.size() - pos);
          pos = buf.size();
          if (!out.empty() && out.back() == '\r') out.pop_back();
          return true;
        }
        return false;
      }
      if (pos > (1 << 20)) {
        buf.erase(0, pos);
        pos = 0;
      }
    }
  };
  char esc = '\\';
  bool directives_open = true;
  bool first_physical = true;
  std::string result;
  std::string phys;
  while (next_line(phys)) {
    if (too_long) break;
    if (first_physical) {
      first_physical = false;
      if (phys.size() >= 3 && (unsigned char)phys[0] == 0xEF && (unsigned char)phys[1] == 0xBB && (unsigned char)phys[2] == 0xBF)
        phys.erase(0, 3);
    }
    std::string line = ltrim(phys);
    if (directives_open) {
      // parser directives: "# escape=`" / "# syntax=..." before anything else
      if (!line.empty() && line[0] == '#') {
        std::string body = ltrim(line.substr(1));
        std::string key;
        size_t i = 0;
        while (i < body.size() && (isalnum((unsigned char)body[i]) || body[i] == '_')) key += (char)tolower((unsigned char)body[i++]);
        size_t j = i;
        while (j < body.size() && (body[j] == ' ' || body[j] == '\t')) j++;
        if (!key.empty() && j < body.size() && body[j] == '=') {
          std::string val = ltrim(body.substr(j + 1));
          while (!val.empty() && is_space((unsigned char)val.back())) val.pop_back();
          if (key == "escape" && (val == "`" || val == "\\")) esc = val[0];
          continue;
        }
        directives_open = false;
      } else if (!line.empty()) {
        directives_open = false;
      }
    }
    if (line.empty() || line[0] == '#') continue;
    bool cont = trim_continuation(line, esc);
    while (cont) {
      std::string nxt;
      if (!next_line(nxt) || too_long) {
        cont = false;
        break;
      }
      std::string t = ltrim(nxt);
      if (!t.empty() && t[0] == '#') continue;  // comment inside continuation
      if (t.empty()) continue;                   // empty continuation line
      cont = trim_continuation(nxt, esc);
      line += nxt;
    }
    if (too_long) break;
    std::string cmd = lower_word(line);
    if (cmd == "arg") continue;
    if (cmd == "from") result = line;
    break;
  }
  close(fd);
  if (too_long) return "";
  return result;
}

static std::vector<std::string> sniff_all(const std::vector<std::string> &paths, int nthreads) {
  std::vector<std::string> out(paths.size());
  py::gil_scoped_release nogil;
  if (nthreads <= 1 || paths.size() < 64) {
    for (size_t i = 0; i < paths.size(); i++) out[i] = sniff_one(paths[i]);
    return out;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  int nt = std::min<int>(nthreads, (int)((paths.size() + 31) / 32));
  for (int t = 0; t < nt; t++) {
    pool.emplace_back([&]() {
      for (;;) {
        size_t i = next.fetch_add(1);
        if (i >= paths.size()) break;
        out[i] = sniff_one(paths[i]);
      }
    });
  }
  for (auto &th : pool) th.join();
  return out;
}

// FROM lines are file bytes: decoded as UTF-8 with surrogateescape, like the
// Python sniffer (dockerfile_parser.py:sniff_first_from), so a Latin-1 byte in
// one Dockerfile does not fail the whole batch.
py::list sniff_dockerfiles(const std::vector<std::string> &paths, int nthreads) {
  std::vector<std::string> raw = sniff_all(paths, nthreads);
  py::list out(raw.size());
  for (size_t i = 0; i < raw.size(); i++) {
    PyObject *o = PyUnicode_DecodeUTF8(raw[i].data(), static_cast<Py_ssize_t>(raw[i].size()), "surrogateescape");
    if (!o) throw py::error_already_set();
    out[i] = py::reinterpret_steal<py::str>(o);
  }
  return out;
}

// ----------------------------------------------------------------------------
// hashes
// ----------------------------------------------------------------------------
uint64_t crc_table[256];
bool crc_init = false;

uint64_t crc64_ecma(const py::bytes &b) {
  if (!crc_init) {
    for (int i = 0; i < 256; i++) {
      uint64_t c = (uint64_t)i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xC96C5795D7870F42ULL : (c >> 1);
      crc_table[i] = c;
    }
    crc_init = true;
  }
  std::string s = b;
  uint64_t crc = ~0ULL;
  for (unsigned char c : s) crc = crc_table[(crc ^ c) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

uint64_t fnv64a(const py::bytes &b) {
  std::string s = b;
  uint64_t h = 0xcbf29ce484222325ULL;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x100000001b3ULL;
  }
  return h;
}

// ----------------------------------------------------------------------------
// Wagner-Fischer (smetrics.WagnerFischer semantics, byte-wise)
// ----------------------------------------------------------------------------
int wf_distance(std::string_view a, std::string_view b, int icost, int dcost, int scost) {
  std::vector<int> row1(b.size() + 1), row2(b.size() + 1);
  for (size_t i = 1; i <= b.size(); i++) row1[i] = (int)i * icost;
  for (size_t i = 1; i <= a.size(); i++) {
    row2[0] = (int)i * dcost;
    for (size_t j = 1; j <= b.size(); j++) {
      if (a[i - 1] == b[j - 1]) {
        row2[j] = row1[j - 1];
      } else {
        int ins = row2[j - 1] + icost, del = row1[j] + dcost, sub = row1[j - 1] + scost;
        if (ins < del && ins < sub) row2[j] = ins;
        else if (del < sub) row2[j] = del;
        else row2[j] = sub;
      }
    }
    std::swap(row1, row2);
  }
  return row1[b.size()];
}

int wagner_fischer(const std::string &a, const std::string &b, int icost, int dcost, int scost) {
  return wf_distance(a, b, icost, dcost, scost);
}

// Borrowed UTF-8 (str) / raw (bytes) buffers of a Python list's items; valid
// while the list is alive.  Avoids copying every item into a std::string
// (200k-item lists cost ~20 ms of pybind11 conversion, more than the search).
std::vector<std::string_view> views_of(const py::list &items) {
  PyObject *lst = items.ptr();
  const Py_ssize_t n = PyList_GET_SIZE(lst);
  std::vector<std::string_view> v((size_t)n);
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject *o = PyList_GET_ITEM(lst, i);
    Py_ssize_t len = 0;
    const char *s;
    if (PyUnicode_Check(o)) {
      s = PyUnicode_AsUTF8AndSize(o, &len);
      if (!s) throw py::error_already_set();
    } else if (PyBytes_Check(o)) {
      s = PyBytes_AS_STRING(o);
      len = PyBytes_GET_SIZE(o);
    } else {
      throw py::type_error("items must be str or bytes");
    }
    v[(size_t)i] = std::string_view(s, (size_t)len);
  }
  return v;
}

// Bit-parallel LCS (Hyyro): with ins=del=1, sub=2 the weighted distance is
// |a| + |b| - 2*LCS(a, b).  The query b is encoded once as per-byte match masks
// over ceil(|b|/64) words; each byte of a then costs ~5 word ops per word.
struct QueryMasks {
  int len = 0, words = 0;
  std::vector<uint64_t> m;  // [256][words]
};

QueryMasks make_masks(std::string_view b) {
  QueryMasks q;
  q.len = (int)b.size();
  q.words = std::max(1, (q.len + 63) / 64);
  q.m.assign((size_t)256 * q.words, 0);
  for (int k = 0; k < q.len; k++) q.m[(size_t)(uint8_t)b[k] * q.words + k / 64] |= (1ULL << (k % 64));
  return q;
}

int lcs_distance(std::string_view a, const QueryMasks &q, std::vector<uint64_t> &V) {
  const int W = q.words;
  if (W == 1) {
    uint64_t v = ~0ULL;
    for (unsigned char ch : a) {
      const uint64_t u = v & q.m[ch];
      v = (v + u) | (v - u);
    }
    const uint64_t mask = q.len >= 64 ? ~0ULL : ((1ULL << q.len) - 1ULL);
    return (int)a.size() + q.len - 2 * __builtin_popcountll(~v & mask);
  }
  V.assign(W, ~0ULL);
  for (unsigned char ch : a) {
    const uint64_t *M = &q.m[(size_t)ch * W];
    unsigned carry = 0;
    for (int w = 0; w < W; w++) {
      const uint64_t v = V[w], u = v & M[w];
      const uint64_t sum1 = v + u;
      const unsigned c1 = sum1 < v;
      const uint64_t sum = sum1 + carry;
      const unsigned c2 = sum < sum1;
      carry = c1 | c2;
      V[w] = sum | (v - u);
    }
  }
  int lcs = 0;
  for (int w = 0; w < W; w++) {
    const int bits = std::min(64, q.len - 64 * w);
    const uint64_t mask = bits >= 64 ? ~0ULL : ((1ULL << bits) - 1ULL);
    lcs += __builtin_popcountll(~V[w] & mask);
  }
  return (int)a.size() + q.len - 2 * lcs;
}

template <class F>
void parallel_for(size_t n, int nthreads, size_t grain, F f) {
  if (nthreads <= 1 || n < grain) {
    if (n) f(0, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    const size_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo >= hi) break;
    pool.emplace_back(f, lo, hi);
  }
  for (auto &th : pool) th.join();
}

// Threads worth starting for `pairs` LCS evaluations: each thread gets at
// least ~16k pairs (~0.3 ms), so small batches never pay thread start-up
// (16 threads for 1.6k pairs cost 0.49 ms vs ~0.04 ms on one thread, MI355X host).
static int threads_for(size_t pairs, int nthreads) {
  const size_t t = pairs / 16384;
  return (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, nthreads), t));
}

// distance matrix [len(as) x len(bs)] as an int32 numpy array
py::array_t<int32_t> edit_distance_batch(const py::list &as_list, const py::list &bs_list, int icost, int dcost,
                                         int scost, int nthreads) {
  const std::vector<std::string_view> as = views_of(as_list), bs = views_of(bs_list);
  const size_t na = as.size(), nb = bs.size();
  py::array_t<int32_t> arr({na, nb});
  int32_t *out = arr.mutable_data();
  const bool lcs = (icost == 1 && dcost == 1 && scost == 2);
  {
    py::gil_scoped_release nogil;
    if (lcs) {
      std::vector<QueryMasks> qm(nb);
      for (size_t j = 0; j < nb; j++) qm[j] = make_masks(bs[j]);
      parallel_for(na, threads_for(na * nb, nthreads), 1, [&](size_t lo, size_t hi) {
        std::vector<uint64_t> V;
        for (size_t i = lo; i < hi; i++)
          for (size_t j = 0; j < nb; j++) out[i * nb + j] = lcs_distance(as[i], qm[j], V);
      });
    } else {
      parallel_for(na * nb, nthreads, 4096, [&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; k++) out[k] = wf_distance(as[k / nb], bs[k % nb], icost, dcost, scost);
      });
    }
  }
  return arr;
}

// Pack a list of str/bytes into one buffer + int64 offsets[n+1] (the layout the
// GPU kernel library consumes), without building n Python bytes objects.
// Pack str/bytes items back to back: (bytes, int64 offsets[n+1], max length).
// Two passes over borrowed list items; the result bytes object is filled in place.
std::tuple<py::bytes, py::array_t<int64_t>, int64_t> pack_strings(const py::list &items) {
  PyObject *lst = items.ptr();
  const Py_ssize_t n = PyList_GET_SIZE(lst);
  py::array_t<int64_t> off(n + 1);
  int64_t *po = off.mutable_data();
  std::vector<const char *> ptrs((size_t)n);
  po[0] = 0;
  int64_t maxlen = 0;
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject *o = PyList_GET_ITEM(lst, i);
    Py_ssize_t len = 0;
    const char *s;
    if (PyUnicode_Check(o)) {
      s = PyUnicode_AsUTF8AndSize(o, &len);  // O(1) for ASCII strings
      if (!s) throw py::error_already_set();
    } else if (PyBytes_Check(o)) {
      s = PyBytes_AS_STRING(o);
      len = PyBytes_GET_SIZE(o);
    } else {
      throw py::type_error("pack_strings: items must be str or bytes");
    }
    ptrs[(size_t)i] = s;
    po[i + 1] = po[i] + (int64_t)len;
    if (len > maxlen) maxlen = len;
  }
  PyObject *b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)po[n]);
  if (!b) throw py::error_already_set();
  char *dst = PyBytes_AS_STRING(b);
  for (Py_ssize_t i = 0; i < n; i++) memcpy(dst + po[i], ptrs[(size_t)i], (size_t)(po[i + 1] - po[i]));
  return std::make_tuple(py::reinterpret_steal<py::bytes>(b), off, maxlen);
}

// For every query: (first index of the minimum distance, that distance); (-1, -1) without options.
// Runs without the GIL; pi/pd have nb entries.
static void closest_core(const std::vector<std::string_view> &as, const std::vector<std::string_view> &bs,
                         int nthreads, int32_t *pi, int32_t *pd) {
  const size_t na = as.size(), nb = bs.size();
  {
    const int nt = threads_for(na * nb, nthreads);
    std::vector<QueryMasks> qm(nb);
    for (size_t j = 0; j < nb; j++) qm[j] = make_masks(bs[j]);
    if (nb >= (size_t)nt * 2 || nt == 1) {
      // enough queries: split them
      parallel_for(nb, nt, 1, [&](size_t lo, size_t hi) {
        std::vector<uint64_t> V;
        for (size_t j = lo; j < hi; j++) {
          int bi = -1, bd = -1;
          for (size_t i = 0; i < na; i++) {
            const int d = lcs_distance(as[i], qm[j], V);
            if (bi < 0 || d < bd) bi = (int)i, bd = d;
          }
          pi[j] = bi;
          pd[j] = bd;
        }
      });
    } else {
      // few queries, many options: split the options, merge per query in range
      // order so ties still resolve to the first index
      const size_t chunk = (na + nt - 1) / nt;
      std::vector<int> pbi((size_t)nt * nb, -1), pbd((size_t)nt * nb, -1);
      parallel_for((size_t)nt, nt, 1, [&](size_t tlo, size_t thi) {
        std::vector<uint64_t> V;
        for (size_t t = tlo; t < thi; t++) {
          const size_t lo = t * chunk, hi = std::min(na, lo + chunk);
          for (size_t j = 0; j < nb; j++) {
            int bi = -1, bd = -1;
            for (size_t i = lo; i < hi; i++) {
              const int d = lcs_distance(as[i], qm[j], V);
              if (bi < 0 || d < bd) bi = (int)i, bd = d;
            }
            pbi[t * nb + j] = bi;
            pbd[t * nb + j] = bd;
          }
        }
      });
      for (size_t j = 0; j < nb; j++) {
        int bi = -1, bd = -1;
        for (int t = 0; t < nt; t++) {
          const int i = pbi[(size_t)t * nb + j], d = pbd[(size_t)t * nb + j];
          if (i >= 0 && (bi < 0 || d < bd)) bi = i, bd = d;
        }
        pi[j] = bi;
        pd[j] = bd;
      }
    }
  }
}

std::pair<py::array_t<int32_t>, py::array_t<int32_t>> closest_batch(const py::list &as_list, const py::list &bs_list,
                                                                    int nthreads) {
  const std::vector<std::string_view> as = views_of(as_list), bs = views_of(bs_list);
  py::array_t<int32_t> idx(bs.size()), dist(bs.size());
  int32_t *pi = idx.mutable_data(), *pd = dist.mutable_data();
  {
    py::gil_scoped_release nogil;
    closest_core(as, bs, nthreads, pi, pd);
  }
  return {idx, dist};
}

// Same as closest_batch with plain lists: the CLI's handful of fuzzy matches
// (collect -a cf) then never imports numpy, which costs more than the matching.
std::pair<py::list, py::list> closest_list(const py::list &as_list, const py::list &bs_list, int nthreads) {
  const std::vector<std::string_view> as = views_of(as_list), bs = views_of(bs_list);
  std::vector<int32_t> vi(bs.size()), vd(bs.size());
  {
    py::gil_scoped_release nogil;
    closest_core(as, bs, nthreads, vi.data(), vd.data());
  }
  py::list li(bs.size()), ld(bs.size());
  for (size_t j = 0; j < bs.size(); j++) {
    li[j] = py::int_(vi[j]);
    ld[j] = py::int_(vd[j]);
  }
  return {li, ld};
}

// ----------------------------------------------------------------------------
// bounded-parallel process pool
// ----------------------------------------------------------------------------
struct Child {
  pid_t pid = -1;
  int outfd = -1;
  size_t idx = 0;
  std::string out;
  bool done_reading = false;
  double start = 0;
  bool killed = false;
};

double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Runs argv[i] with working directory cwd[i]; stdout captured, stderr inherited
// (the reference wires detector stderr to the console).  At most `parallel`
// children run at once.  Returns (exit_code, stdout) per command; exit code
// -1 means spawn failure, -2 timeout.
std::vector<std::pair<int, py::bytes>> run_commands(const std::vector<std::vector<std::string>> &argvs,
                                                     const std::vector<std::string> &cwds, int parallel,
                                                     double timeout_s) {
  std::vector<int> codes(argvs.size(), -1);
  std::vector<std::string> outs(argvs.size());
  {
    py::gil_scoped_release nogil;
    if (parallel < 1) parallel = 1;
    std::vector<Child> running;
    size_t next = 0;
    auto spawn = [&](size_t i) -> bool {
      int pfd[2];
      if (pipe2(pfd, O_CLOEXEC) != 0) return false;
      posix_spawn_file_actions_t fa;
      posix_spawn_file_actions_init(&fa);
      posix_spawn_file_actions_adddup2(&fa, pfd[1], 1);
      int devnull = -1;
      (void)devnull;
      posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
#if defined(__GLIBC__) && (__GLIBC__ > 2 || (__GLIBC__ == 2 && __GLIBC_MINOR__ >= 29))
      if (!cwds[i].empty()) posix_spawn_file_actions_addchdir_np(&fa, cwds[i].c_str());
#endif
      std::vector<char *> argv;
      for (auto &s : argvs[i]) argv.push_back(const_cast<char *>(s.c_str()));
      argv.push_back(nullptr);
      pid_t pid;
      int rc = posix_spawnp(&pid, argv[0], &fa, nullptr, argv.data(), environ);
      posix_spawn_file_actions_destroy(&fa);
      close(pfd[1]);
      if (rc != 0) {
        close(pfd[0]);
        return false;
      }
      Child c;
      c.pid = pid;
      c.outfd = pfd[0];
      c.idx = i;
      c.start = now_s();
      running.push_back(std::move(c));
      return true;
    };
    while (next < argvs.size() || !running.empty()) {
      while ((int)running.size() < parallel && next < argvs.size()) {
        size_t i = next++;
        if (!spawn(i)) codes[i] = -1;
      }
      if (running.empty()) continue;
      std::vector<struct pollfd> pfds;
      for (auto &c : running) pfds.push_back({c.done_reading ? -1 : c.outfd, POLLIN, 0});
      int pr = poll(pfds.data(), pfds.size(), 50);
      (void)pr;
      for (size_t k = 0; k < running.size(); k++) {
        Child &c = running[k];
        if (!c.done_reading && (pfds[k].revents & (POLLIN | POLLHUP | POLLERR))) {
          char buf[8192];
          ssize_t n = read(c.outfd, buf, sizeof(buf));
          if (n > 0) c.out.append(buf, (size_t)n);
          else c.done_reading = true;
        }
        if (!c.killed && timeout_s > 0 && now_s() - c.start > timeout_s) {
          kill(c.pid, SIGKILL);
          c.killed = true;
        }
      }
      // reap finished children whose output is drained
      for (size_t k = 0; k < running.size();) {
        Child &c = running[k];
        if (c.done_reading) {
          int status = 0;
          pid_t w = waitpid(c.pid, &status, c.killed ? 0 : WNOHANG);
          if (w == c.pid) {
            close(c.outfd);
            int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
            if (c.killed) code = -2;
            codes[c.idx] = code;
            outs[c.idx] = std::move(c.out);
            running.erase(running.begin() + k);
            continue;
          }
        }
        k++;
      }
    }
  }
  std::vector<std::pair<int, py::bytes>> res;
  res.reserve(argvs.size());
  for (size_t i = 0; i < argvs.size(); i++) res.emplace_back(codes[i], py::bytes(outs[i]));
  return res;
}

}  // namespace

// ---------------------------------------------------------------------------
// Batched output writes: open(O_TRUNC) + write + fchmod(mode) per file, with
// the GIL released; different directories are written by different threads.  Returns errno per file (0 = ok).  A path
// listed twice keeps its last content (written once, like sequential writes).
// ---------------------------------------------------------------------------
// ioutil.WriteFile(path, data, perm): a new file gets perm & ~umask, an
// existing one is truncated and keeps its permissions (no chmod).
static int write_one(const std::string &path, const std::string &data, int mode) {
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, static_cast<mode_t>(mode));
  if (fd < 0) return errno;
  const char *p = data.data();
  size_t left = data.size();
  while (left) {
    ssize_t w = ::write(fd, p, left);
    if (w < 0) {
      if (errno == EINTR) continue;
      int e = errno;
      ::close(fd);
      return e;
    }
    p += w;
    left -= static_cast<size_t>(w);
  }
  if (::close(fd) != 0) return errno;
  return 0;
}

static constexpr size_t kParallelWriteMin = 512;

std::vector<int> write_files(const std::vector<std::string> &paths, const std::vector<py::bytes> &datas,
                             const std::vector<int> &modes, int nthreads) {
  const size_t n = paths.size();
  if (datas.size() != n || modes.size() != n) throw std::invalid_argument("paths, datas and modes differ in length");
  std::vector<std::string> bufs(n);
  for (size_t i = 0; i < n; i++) bufs[i] = static_cast<std::string>(datas[i]);
  std::vector<int> err(n, 0);
  std::vector<char> skip(n, 0);  // superseded by a later write to the same path
  {
    std::vector<size_t> order(n);
    for (size_t i = 0; i < n; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return paths[a] < paths[b]; });
    for (size_t k = 0; k + 1 < n; k++)
      if (paths[order[k]] == paths[order[k + 1]]) skip[order[k]] = 1;
  }
  // Creating entries in one directory serialises on that directory's inode
  // lock (threads only add contention), so work is split by parent directory.
  std::map<std::string, std::vector<size_t>> by_dir;
  for (size_t i = 0; i < n; i++)
    if (!skip[i]) by_dir[paths[i].substr(0, paths[i].rfind('/') + 1)].push_back(i);
  std::vector<const std::vector<size_t> *> groups;
  for (auto &kv : by_dir) groups.push_back(&kv.second);
  // A command's output (a hundred-odd small files) is written faster by this
  // thread alone than by starting workers, whose first start in a process
  // also pays for fresh thread stacks; threads only pay off on big batches.
  if (n < kParallelWriteMin) nthreads = 1;
  {
    py::gil_scoped_release nogil;
    parallel_for(groups.size(), std::min<int>(nthreads, static_cast<int>(groups.size())), 2, [&](size_t lo, size_t hi) {
      for (size_t g = lo; g < hi; g++)
        for (size_t i : *groups[g]) err[i] = write_one(paths[i], bufs[i], modes[i]);
    });
  }
  return err;
}

// ---------------------------------------------------------------------------
// remove_tree: RemoveAll(out) without Python per-entry overhead.  Depth-first
// with openat/unlinkat relative to directory fds; symlinks are unlinked, never
// followed.  Returns (errno, path) of the first failure, (0, "") on success.
// ---------------------------------------------------------------------------
static int remove_dir_contents(int dfd, const std::string &path, std::string &errpath) {
  DIR *d = fdopendir(dfd);
  if (!d) {
    errpath = path;
    int e = errno;
    ::close(dfd);
    return e;
  }
  int err = 0;
  std::vector<std::pair<std::string, bool>> entries;
  while (struct dirent *de = readdir(d)) {
    const char *n = de->d_name;
    if (n[0] == '.' && (n[1] == 0 || (n[1] == '.' && n[2] == 0))) continue;
    bool isdir;
    if (de->d_type == DT_DIR) {
      isdir = true;
    } else if (de->d_type == DT_UNKNOWN) {
      struct stat st;
      isdir = fstatat(dirfd(d), n, &st, AT_SYMLINK_NOFOLLOW) == 0 && S_ISDIR(st.st_mode);
    } else {
      isdir = false;
    }
    entries.emplace_back(n, isdir);
  }
  for (auto &e : entries) {
    if (err) break;
    if (e.second) {
      int cfd = openat(dirfd(d), e.first.c_str(), O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
      if (cfd < 0) {
        err = errno;
        errpath = path + "/" + e.first;
        break;
      }
      err = remove_dir_contents(cfd, path + "/" + e.first, errpath);
      if (!err && unlinkat(dirfd(d), e.first.c_str(), AT_REMOVEDIR) != 0) {
        err = errno;
        errpath = path + "/" + e.first;
      }
    } else if (unlinkat(dirfd(d), e.first.c_str(), 0) != 0) {
      err = errno;
      errpath = path + "/" + e.first;
    }
  }
  closedir(d);  // closes dfd
  return err;
}

std::pair<int, py::bytes> remove_tree(const std::string &path) {
  std::string errpath;
  int err = 0;
  {
    py::gil_scoped_release nogil;
    struct stat st;
    if (lstat(path.c_str(), &st) != 0) {
      err = errno;
      errpath = path;
    } else if (!S_ISDIR(st.st_mode)) {
      if (unlink(path.c_str()) != 0) err = errno, errpath = path;
    } else {
      int fd = open(path.c_str(), O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
      if (fd < 0) {
        err = errno;
        errpath = path;
      } else {
        err = remove_dir_contents(fd, path, errpath);
        if (!err && rmdir(path.c_str()) != 0) err = errno, errpath = path;
      }
    }
  }
  return {err, py::bytes(errpath)};  // raw bytes: the caller decodes with os.fsdecode
}

// yaml_emit.cpp
extern "C" PyObject* m2k_yaml_dump(PyObject* data, int sort_maps, PyObject* gomap, PyObject* scalar_fn,
                                   PyObject* style_fn, PyObject* sort_fn);

static py::str yaml_dump(py::object data, bool sort_maps, py::object gomap, py::object scalar_fn, py::object style_fn,
                         py::object sort_fn) {
  PyObject* r = m2k_yaml_dump(data.ptr(), sort_maps ? 1 : 0, gomap.ptr(), scalar_fn.ptr(), style_fn.ptr(), sort_fn.ptr());
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::str>(r);
}

extern "C" PyObject* m2k_yaml_load(PyObject* text, int mode, int multi, PyObject* resolve_number,
                                   PyObject* unsupported);

static py::object yaml_load(py::object text, int mode, bool multi, py::object resolve_number, py::object unsupported) {
  PyObject* r = m2k_yaml_load(text.ptr(), mode, multi ? 1 : 0, resolve_number.ptr(), unsupported.ptr());
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

extern "C" PyObject* m2k_schema_init(PyObject* structs, PyObject* fallback);
extern "C" PyObject* m2k_schema_marshal(PyObject* obj, PyObject* type_name);

static py::object schema_init(py::object structs, py::object fallback) {
  PyObject* r = m2k_schema_init(structs.ptr(), fallback.ptr());
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

static py::object schema_marshal(py::object obj, py::object type_name) {
  PyObject* r = m2k_schema_marshal(obj.ptr(), type_name.ptr());
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

extern "C" PyObject* m2k_proc_spawn(PyObject* argv, PyObject* cwd, long out_mode, long err_mode);
extern "C" PyObject* m2k_proc_wait(long pid, long out_fd, long err_fd, double timeout_s);

extern "C" PyObject* m2k_procgroup_new();
extern "C" PyObject* m2k_procgroup_add(PyObject* cap, long key, long pid, long out_fd, long err_fd, double timeout_s);
extern "C" PyObject* m2k_procgroup_wait_any(PyObject* cap);

static py::object steal_or_throw(PyObject* r) {
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

static py::object procgroup_new() { return steal_or_throw(m2k_procgroup_new()); }
static py::object procgroup_add(py::object g, long key, long pid, long out_fd, long err_fd, double timeout_s) {
  return steal_or_throw(m2k_procgroup_add(g.ptr(), key, pid, out_fd, err_fd, timeout_s));
}
static py::object procgroup_wait_any(py::object g) { return steal_or_throw(m2k_procgroup_wait_any(g.ptr())); }

static py::object proc_spawn(py::object argv, py::object cwd, long out_mode, long err_mode) {
  PyObject* r = m2k_proc_spawn(argv.ptr(), cwd.ptr(), out_mode, err_mode);
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

static py::object proc_wait(long pid, long out_fd, long err_fd, double timeout_s) {
  PyObject* r = m2k_proc_wait(pid, out_fd, err_fd, timeout_s);
  if (!r) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

PYBIND11_MODULE(_m2k_native, m) {
  m.doc() = "move2kube_amd native runtime (walk, sniff, spawn pool, hashes, edit distance)";
  m.def("walk", &walk, py::arg("root"));
  m.def("sniff_dockerfiles", &sniff_dockerfiles, py::arg("paths"), py::arg("nthreads") = 8);
  m.def("crc64_ecma", &crc64_ecma);
  m.def("fnv64a", &fnv64a);
  m.def("wagner_fischer", &wagner_fischer, py::arg("a"), py::arg("b"), py::arg("icost") = 1, py::arg("dcost") = 1,
        py::arg("scost") = 2);
  m.def("edit_distance_batch", &edit_distance_batch, py::arg("as"), py::arg("bs"), py::arg("icost") = 1,
        py::arg("dcost") = 1, py::arg("scost") = 2, py::arg("nthreads") = 8);
  m.def("pack_strings", &pack_strings, py::arg("items"));
  m.def("closest_batch", &closest_batch, py::arg("as"), py::arg("bs"), py::arg("nthreads") = 8);
  m.def("closest_list", &closest_list, py::arg("as"), py::arg("bs"), py::arg("nthreads") = 8);
  m.def("remove_tree", &remove_tree, py::arg("path"));
  m.def("write_files", &write_files, py::arg("paths"), py::arg("datas"), py::arg("modes"), py::arg("nthreads") = 8);
  m.def("yaml_dump", &yaml_dump, py::arg("data"), py::arg("sort_maps"), py::arg("gomap"), py::arg("scalar_fn"),
        py::arg("style_fn"), py::arg("sort_fn"));
  m.def("yaml_load", &yaml_load, py::arg("text"), py::arg("mode"), py::arg("multi"), py::arg("resolve_number"),
        py::arg("unsupported"));
  m.def("schema_init", &schema_init, py::arg("structs"), py::arg("fallback"));
  m.def("schema_marshal", &schema_marshal, py::arg("obj"), py::arg("type_name"));
  m.def("proc_spawn", &proc_spawn, py::arg("argv"), py::arg("cwd"), py::arg("stdout"), py::arg("stderr"));
  m.def("proc_wait", &proc_wait, py::arg("pid"), py::arg("out_fd"), py::arg("err_fd"), py::arg("timeout_s"));
  m.def("procgroup_new", &procgroup_new);
  m.def("procgroup_add", &procgroup_add, py::arg("group"), py::arg("key"), py::arg("pid"), py::arg("out_fd"),
        py::arg("err_fd"), py::arg("timeout_s"));
  m.def("procgroup_wait_any", &procgroup_wait_any, py::arg("group"));
  m.def("run_commands", &run_commands, py::arg("argvs"), py::arg("cwds"), py::arg("parallel") = 8,
        py::arg("timeout_s") = 0.0);
}
