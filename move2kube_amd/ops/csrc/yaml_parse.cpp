// Native YAML loader for the documents move2kube reads on every command:
// compose files, CF manifests, plans, QA caches, cluster metadata, Kubernetes
// manifests.  The reference decodes them with go-yaml (compiled Go); this is
// the MI355X host's native equivalent of that decode step, so a CLI process no
// longer has to import and initialise PyYAML (whose resolver regexes alone cost
// more than the parse) just to read a plan.
//
// Design: a strict, line-oriented recursive-descent parser for the block-style
// subset those files use - block mappings and sequences (including compact
// "- key: v" and same-indent "key:\n- item" forms), plain / single-quoted /
// double-quoted single-line scalars, literal and folded block scalars
// (chomping and indentation indicators, libyaml's folding algorithm), single-
// line flow collections, comments and multi-document streams.  Scalars are
// resolved exactly like yamlio's three PyYAML loader classes (go-yaml v3 typed,
// go-yaml v2 typed, raw); numbers go through the Python `resolve_number`
// callable (yamlio.go_resolve_number), so both paths share one definition.
//
// Anything outside the subset - anchors/aliases/tags, merge keys, explicit
// keys, directives, tabs, multi-line plain/quoted scalars or flow collections,
// unusual characters, and every malformed document - makes the parser return
// the `unsupported` sentinel, and yamlio falls back to PyYAML.  So the subset
// never has to reproduce an error message, and an input is either decoded
// identically (tests/test_yaml_native.py checks this differentially against
// the PyYAML loaders, on fixtures and generated documents) or not at all.

#include <Python.h>

#include <cstring>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

namespace m2kyamlp {

struct Unsupported {};
struct PyErrorSet {};
// Nesting past go-yaml's limit (yaml.v3 scannerc.go max_flow_level /
// max_indents = 10000): a parse error of this document, never handed to
// PyYAML, whose C composer recurses once per level and overflows the stack.
struct TooDeep {};
constexpr int kMaxDepth = 10000;
// libyaml / go-yaml refuse a simple (implicit) key longer than 1024 characters;
// bytes >= characters, so a longer byte span is left to PyYAML to judge.
constexpr int kMaxSimpleKey = 1024;

enum Mode { TYPED = 0, V2 = 1, RAW = 2 };

// owning PyObject* holder
class Ref {
 public:
  Ref() : p_(nullptr) {}
  explicit Ref(PyObject* p) : p_(p) {
    if (!p_) throw PyErrorSet();
  }
  Ref(const Ref&) = delete;
  Ref& operator=(const Ref&) = delete;
  Ref(Ref&& o) noexcept : p_(o.p_) { o.p_ = nullptr; }
  Ref& operator=(Ref&& o) noexcept {
    if (this != &o) {
      Py_XDECREF(p_);
      p_ = o.p_;
      o.p_ = nullptr;
    }
    return *this;
  }
  ~Ref() { Py_XDECREF(p_); }
  PyObject* get() const { return p_; }
  PyObject* release() {
    PyObject* p = p_;
    p_ = nullptr;
    return p;
  }

 private:
  PyObject* p_;
};

struct Line {
  const char* s;  // start of the line
  int len;        // bytes, without the line break (and a '\r' before it)
  int indent;     // leading spaces
  bool content;   // not blank and not a comment line
  bool has_break; // terminated by a line break (false only for the last line)
};

static inline bool is_flow_ind(char c) { return c == ',' || c == '[' || c == ']' || c == '{' || c == '}'; }

class Parser {
  // one level of node_at / flow recursion
  struct DepthGuard {
    int& d;
    explicit DepthGuard(int& depth) : d(depth) {
      if (++d > kMaxDepth) {
        --d;
        throw TooDeep();
      }
    }
    ~DepthGuard() { --d; }
  };
  int depth_ = 0;

 public:
  Parser(const char* s, size_t n, int mode, PyObject* resolve_number)
      : mode_(mode), resolve_number_(resolve_number) {
    split(s, n);
  }

  // the documents of the stream
  std::vector<Ref> stream() {
    std::vector<Ref> docs;
    size_t li = 0;
    bool need_marker = false;  // after "..." only "---" or the end may follow
    for (;;) {
      li = next_content(li);
      if (li >= L_.size()) break;
      const Line& ln = L_[li];
      if (ln.len > 0 && ln.s[0] == '%') throw Unsupported();
      if (is_marker(ln, '-')) {
        rest_is_blank(ln, 3);
        li = next_content(li + 1);
        if (li >= L_.size() || is_marker(L_[li], '-')) {
          docs.emplace_back(none());
          need_marker = false;
          continue;
        }
        if (is_marker(L_[li], '.')) {
          rest_is_blank(L_[li], 3);
          docs.emplace_back(none());
          li++;
          need_marker = true;
          continue;
        }
      } else if (is_marker(ln, '.') || need_marker) {
        throw Unsupported();
      }
      li_ = li;
      const Line& first = L_[li_];
      Ref root(node_at(first.indent, -1, true));
      docs.push_back(std::move(root));
      li = next_content(li_);
      need_marker = false;
      if (li < L_.size()) {
        if (is_marker(L_[li], '.')) {
          rest_is_blank(L_[li], 3);
          li++;
          need_marker = true;
        } else if (!is_marker(L_[li], '-')) {
          throw Unsupported();
        }
      }
    }
    return docs;
  }

 private:
  std::vector<Line> L_;
  size_t li_ = 0;  // current line
  int mode_;
  PyObject* resolve_number_;

  // ---- input --------------------------------------------------------------
  void split(const char* s, size_t n) {
    const unsigned char* u = reinterpret_cast<const unsigned char*>(s);
    for (size_t i = 0; i < n; i++) {
      const unsigned char c = u[i];
      if (c < 0x20) {
        if (c == '\n') continue;
        if (c == '\r' && i + 1 < n && u[i + 1] == '\n') continue;
        throw Unsupported();  // tabs, lone CR, control characters
      }
      if (c == 0x7f) throw Unsupported();
      if (c == 0xC2 && i + 1 < n && u[i + 1] >= 0x80 && u[i + 1] <= 0x9F) throw Unsupported();  // C1, NEL
      if (c == 0xE2 && i + 2 < n && u[i + 1] == 0x80 && (u[i + 2] == 0xA8 || u[i + 2] == 0xA9))
        throw Unsupported();  // LS, PS line breaks
      if (c == 0xEF && i + 2 < n &&
          ((u[i + 1] == 0xBB && u[i + 2] == 0xBF) || (u[i + 1] == 0xBF && (u[i + 2] == 0xBE || u[i + 2] == 0xBF))))
        throw Unsupported();  // BOM, U+FFFE/FFFF
    }
    size_t i = 0;
    while (i < n) {
      size_t j = i;
      while (j < n && s[j] != '\n') j++;
      Line ln;
      ln.s = s + i;
      size_t len = j - i;
      if (len && s[i + len - 1] == '\r') len--;
      ln.len = (int)len;
      ln.has_break = j < n;
      int k = 0;
      while (k < ln.len && ln.s[k] == ' ') k++;
      ln.indent = k;
      ln.content = k < ln.len && ln.s[k] != '#';
      L_.push_back(ln);
      i = j + 1;
    }
  }

  size_t next_content(size_t li) const {
    while (li < L_.size() && !L_[li].content) li++;
    return li;
  }

  static bool is_marker(const Line& ln, char c) {
    return ln.len >= 3 && ln.s[0] == c && ln.s[1] == c && ln.s[2] == c && (ln.len == 3 || ln.s[3] == ' ');
  }

  // only spaces and an optional comment from `pos` (a '#' needs a space before it)
  static void rest_is_blank(const Line& ln, int pos) {
    int p = pos;
    while (p < ln.len && ln.s[p] == ' ') p++;
    if (p >= ln.len) return;
    if (ln.s[p] == '#' && p > pos) return;
    if (ln.s[p] == '#' && pos > 0 && ln.s[pos - 1] == ' ') return;
    throw Unsupported();
  }

  // ---- scalars ------------------------------------------------------------
  PyObject* none() {
    Py_INCREF(Py_None);
    return Py_None;
  }

  static PyObject* str(const char* p, size_t n) {
    PyObject* o = PyUnicode_DecodeUTF8(p, (Py_ssize_t)n, "strict");
    if (!o) throw PyErrorSet();
    return o;
  }

  static bool eq(const char* p, size_t n, const char* w) { return strlen(w) == n && memcmp(p, w, n) == 0; }

  static bool is_null(const char* p, size_t n) {
    return n == 0 || eq(p, n, "~") || eq(p, n, "null") || eq(p, n, "Null") || eq(p, n, "NULL");
  }

  // -1: not a bool word of the mode
  int bool_word(const char* p, size_t n) const {
    static const char* const t3[] = {"true", "True", "TRUE"};
    static const char* const f3[] = {"false", "False", "FALSE"};
    static const char* const t2[] = {"y", "Y", "yes", "Yes", "YES", "on", "On", "ON"};
    static const char* const f2[] = {"n", "N", "no", "No", "NO", "off", "Off", "OFF"};
    for (const char* w : t3)
      if (eq(p, n, w)) return 1;
    for (const char* w : f3)
      if (eq(p, n, w)) return 0;
    if (mode_ == V2) {
      for (const char* w : t2)
        if (eq(p, n, w)) return 1;
      for (const char* w : f2)
        if (eq(p, n, w)) return 0;
    }
    return -1;
  }

  // implicit resolution of a plain scalar (yamlio._Loaders)
  PyObject* plain(const char* p, size_t n) {
    if (is_null(p, n)) return none();
    if (mode_ == RAW) return str(p, n);
    const int b = bool_word(p, n);
    if (b >= 0) {
      PyObject* o = b ? Py_True : Py_False;
      Py_INCREF(o);
      return o;
    }
    const char c = p[0];
    if (c == '-' || c == '+' || c == '.' || (c >= '0' && c <= '9')) {
      Ref s(str(p, n));
      PyObject* r = PyObject_CallFunctionObjArgs(resolve_number_, s.get(), nullptr);
      if (!r) throw PyErrorSet();
      return r;
    }
    if (n == 2 && p[0] == '<' && p[1] == '<') throw Unsupported();  // merge key
    return str(p, n);
  }

  // first byte of a plain scalar: indicators other than "-?:" + non-space start something else
  static void check_plain_start(const Line& ln, int pos, bool flow) {
    const char c = ln.s[pos];
    if (strchr(",[]{}#&*!|>'\"%@`", c)) throw Unsupported();
    if (c == '-' || c == '?' || c == ':') {
      if (pos + 1 >= ln.len) throw Unsupported();
      const char d = ln.s[pos + 1];
      if (d == ' ' || (flow && is_flow_ind(d))) throw Unsupported();
      if (c != '-') throw Unsupported();  // "?x" / ":x": rare, leave to PyYAML
    }
  }

  // single-line quoted scalar at pos; returns the decoded UTF-8 and sets `end` past the closing quote
  static std::string quoted(const Line& ln, int pos, int& end) {
    std::string out;
    const char q = ln.s[pos];
    int p = pos + 1;
    if (q == '\'') {
      for (;;) {
        if (p >= ln.len) throw Unsupported();  // multi-line
        const char c = ln.s[p];
        if (c == '\'') {
          if (p + 1 < ln.len && ln.s[p + 1] == '\'') {
            out.push_back('\'');
            p += 2;
            continue;
          }
          end = p + 1;
          return out;
        }
        out.push_back(c);
        p++;
      }
    }
    for (;;) {
      if (p >= ln.len) throw Unsupported();
      const char c = ln.s[p];
      if (c == '"') {
        end = p + 1;
        return out;
      }
      if (c != '\\') {
        out.push_back(c);
        p++;
        continue;
      }
      if (p + 1 >= ln.len) throw Unsupported();  // escaped line break
      const char e = ln.s[p + 1];
      p += 2;
      switch (e) {
        case '0': out.push_back('\0'); break;
        case 'a': out.push_back('\x07'); break;
        case 'b': out.push_back('\x08'); break;
        case 't': out.push_back('\x09'); break;
        case 'n': out.push_back('\x0A'); break;
        case 'v': out.push_back('\x0B'); break;
        case 'f': out.push_back('\x0C'); break;
        case 'r': out.push_back('\x0D'); break;
        case 'e': out.push_back('\x1B'); break;
        case ' ': out.push_back(' '); break;
        case '"': out.push_back('"'); break;
        case '/': out.push_back('/'); break;
        case '\\': out.push_back('\\'); break;
        case 'N': append_utf8(out, 0x85); break;
        case '_': append_utf8(out, 0xA0); break;
        case 'L': append_utf8(out, 0x2028); break;
        case 'P': append_utf8(out, 0x2029); break;
        case 'x':
        case 'u':
        case 'U': {
          const int digits = e == 'x' ? 2 : (e == 'u' ? 4 : 8);
          if (p + digits > ln.len) throw Unsupported();
          unsigned long v = 0;
          for (int k = 0; k < digits; k++) {
            const char h = ln.s[p + k];
            int d;
            if (h >= '0' && h <= '9') d = h - '0';
            else if (h >= 'a' && h <= 'f') d = h - 'a' + 10;
            else if (h >= 'A' && h <= 'F') d = h - 'A' + 10;
            else throw Unsupported();
            v = v * 16 + (unsigned long)d;
          }
          p += digits;
          if ((v >= 0xD800 && v <= 0xDFFF) || v > 0x10FFFF) throw Unsupported();
          append_utf8(out, v);
          break;
        }
        default:
          throw Unsupported();
      }
    }
  }

  static void append_utf8(std::string& out, unsigned long v) {
    if (v < 0x80) {
      out.push_back((char)v);
    } else if (v < 0x800) {
      out.push_back((char)(0xC0 | (v >> 6)));
      out.push_back((char)(0x80 | (v & 0x3F)));
    } else if (v < 0x10000) {
      out.push_back((char)(0xE0 | (v >> 12)));
      out.push_back((char)(0x80 | ((v >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (v & 0x3F)));
    } else {
      out.push_back((char)(0xF0 | (v >> 18)));
      out.push_back((char)(0x80 | ((v >> 12) & 0x3F)));
      out.push_back((char)(0x80 | ((v >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (v & 0x3F)));
    }
  }

  // ---- block structure ----------------------------------------------------
  static bool is_seq_entry(const Line& ln, int col) {
    return col < ln.len && ln.s[col] == '-' && (col + 1 == ln.len || ln.s[col + 1] == ' ');
  }

  // If an implicit key starts at pos: its end (exclusive, trimmed) and the
  // position of the ':'; quoted keys are decoded into `qkey`.
  bool key_at(const Line& ln, int pos, int& kend, int& colon, bool& quoted_key, std::string& qkey) const {
    const char c = ln.s[pos];
    if (c == '"' || c == '\'') {
      int end;
      qkey = quoted(ln, pos, end);
      int p = end;
      while (p < ln.len && ln.s[p] == ' ') p++;
      if (p < ln.len && ln.s[p] == ':' && (p + 1 == ln.len || ln.s[p + 1] == ' ')) {
        if (p - pos > kMaxSimpleKey) throw Unsupported();
        kend = end;
        colon = p;
        quoted_key = true;
        return true;
      }
      return false;
    }
    for (int p = pos; p < ln.len; p++) {
      const char d = ln.s[p];
      if (d == '#' && p > pos && ln.s[p - 1] == ' ') return false;  // comment before any ':'
      if (d == ':' && (p + 1 == ln.len || ln.s[p + 1] == ' ')) {
        int e = p;
        while (e > pos && ln.s[e - 1] == ' ') e--;
        if (e == pos) throw Unsupported();  // empty key
        if (p - pos > kMaxSimpleKey) throw Unsupported();
        kend = e;
        colon = p;
        quoted_key = false;
        return true;
      }
    }
    return false;
  }

  // The node starting at (li_, col).  `parent` is the indentation of the
  // enclosing block collection (-1 at the root); `block_ok` is false for a
  // value on its key's line ("key: value"), where block collections cannot start.
  PyObject* node_at(int col, int parent, bool block_ok) {
    DepthGuard guard(depth_);
    const Line& ln = L_[li_];
    const char c = ln.s[col];
    if (is_seq_entry(ln, col)) {
      if (!block_ok) throw Unsupported();
      return block_seq(col);
    }
    if (c == '|' || c == '>') return block_scalar(col, parent);
    if (c == '[' || c == '{') {
      int end;
      Ref v(flow(ln, col, end));
      int p = end;
      while (p < ln.len && ln.s[p] == ' ') p++;
      if (p < ln.len && ln.s[p] == ':') throw Unsupported();  // flow collection as a key
      rest_is_blank(ln, end);
      li_++;
      return v.release();
    }
    int kend, colon;
    bool qk;
    std::string qkey;
    if (key_at(ln, col, kend, colon, qk, qkey)) {
      if (!block_ok) throw Unsupported();  // "key: a: b"
      return block_map(col);
    }
    if (c == '"' || c == '\'') {
      int end;
      std::string v = quoted(ln, col, end);
      rest_is_blank(ln, end);
      li_++;
      return str(v.data(), v.size());
    }
    check_plain_start(ln, col, false);
    // plain scalar up to a comment; a ": " inside would be a mapping value here
    int e = col;
    while (e < ln.len) {
      const char d = ln.s[e];
      if (d == '#' && ln.s[e - 1] == ' ') break;
      if (d == ':' && (e + 1 == ln.len || ln.s[e + 1] == ' ')) throw Unsupported();
      e++;
    }
    while (e > col && ln.s[e - 1] == ' ') e--;
    li_++;
    return plain(ln.s + col, (size_t)(e - col));
  }

  // value of a key or entry whose line ends after the indicator
  PyObject* nested(int parent, bool same_indent_seq) {
    const size_t li = next_content(li_);
    if (li >= L_.size()) return none();
    const Line& ln = L_[li];
    if (is_marker(ln, '-') || is_marker(ln, '.')) return none();
    if (ln.indent > parent) {
      li_ = li;
      return node_at(ln.indent, parent, true);
    }
    if (same_indent_seq && ln.indent == parent && is_seq_entry(ln, parent)) {
      li_ = li;
      return block_seq(parent);
    }
    return none();
  }

  // go-yaml v3 refuses a mapping whose keys repeat (decode.go: same node
  // Kind and Value, i.e. the decoded text of a quoted key or the source text
  // of a plain one).  Such a document is left to the PyYAML path, which
  // reports the keys with their lines (yamlio.py: _duplicate_keys).
  static std::string key_value(PyObject* key, const char* raw, size_t rawlen) {
    if (PyUnicode_Check(key)) {
      Py_ssize_t n = 0;
      const char* u = PyUnicode_AsUTF8AndSize(key, &n);
      if (u) return std::string(u, (size_t)n);
      PyErr_Clear();
    }
    while (rawlen > 0 && raw[rawlen - 1] == ' ') rawlen--;
    return std::string(raw, rawlen);
  }

  static void check_unique(PyObject* d, PyObject* key, std::unordered_set<std::string>& seen, std::string v) {
    int has = PyDict_Contains(d, key);
    if (has < 0) throw PyErrorSet();
    if (has) throw Unsupported();
    if (!seen.insert(std::move(v)).second) throw Unsupported();
  }

  PyObject* block_map(int col) {
    Ref d(PyDict_New());
    std::unordered_set<std::string> seen;
    for (;;) {
      const Line& ln = L_[li_];
      int kend, colon;
      bool qk;
      std::string qkey;
      if (!key_at(ln, col, kend, colon, qk, qkey)) throw Unsupported();
      if (!qk) check_plain_start(ln, col, false);
      Ref key(qk ? str(qkey.data(), qkey.size()) : plain(ln.s + col, (size_t)(kend - col)));
      if (PyObject_Hash(key.get()) == -1) throw PyErrorSet();
      check_unique(d.get(), key.get(), seen, key_value(key.get(), ln.s + col, (size_t)(kend - col)));
      int p = colon + 1;
      while (p < ln.len && ln.s[p] == ' ') p++;
      Ref val;
      if (p >= ln.len || ln.s[p] == '#') {
        li_++;
        val = Ref(nested(col, true));
      } else {
        val = Ref(node_at(p, col, false));
      }
      if (PyDict_SetItem(d.get(), key.get(), val.get()) < 0) throw PyErrorSet();
      const size_t li = next_content(li_);
      if (li >= L_.size()) break;
      const Line& nx = L_[li];
      if (is_marker(nx, '-') || is_marker(nx, '.')) break;
      if (nx.indent < col) break;
      if (nx.indent > col || is_seq_entry(nx, col)) throw Unsupported();
      li_ = li;
    }
    return d.release();
  }

  PyObject* block_seq(int col) {
    Ref lst(PyList_New(0));
    for (;;) {
      const Line& ln = L_[li_];
      int p = col + 1;
      while (p < ln.len && ln.s[p] == ' ') p++;
      Ref item;
      if (p >= ln.len || ln.s[p] == '#') {
        li_++;
        item = Ref(nested(col, false));
      } else {
        item = Ref(node_at(p, col, true));
      }
      if (PyList_Append(lst.get(), item.get()) < 0) throw PyErrorSet();
      const size_t li = next_content(li_);
      if (li >= L_.size()) break;
      const Line& nx = L_[li];
      if (is_marker(nx, '-') || is_marker(nx, '.')) break;
      if (nx.indent < col) break;
      if (nx.indent > col) throw Unsupported();
      if (!is_seq_entry(nx, col)) break;  // a key of the mapping this sequence is the value of
      li_ = li;
    }
    return lst.release();
  }

  // literal/folded block scalar (libyaml yaml_parser_scan_block_scalar)
  PyObject* block_scalar(int col, int parent) {
    const Line& hl = L_[li_];
    const bool literal = hl.s[col] == '|';
    int chomp = 0, incr = 0;
    int p = col + 1;
    for (int k = 0; k < 2 && p < hl.len; k++) {
      const char c = hl.s[p];
      if ((c == '+' || c == '-') && chomp == 0) {
        chomp = c == '+' ? 1 : -1;
        p++;
      } else if (c >= '1' && c <= '9' && incr == 0) {
        incr = c - '0';
        p++;
      } else {
        break;
      }
    }
    if (p < hl.len && hl.s[p] != ' ') throw Unsupported();
    rest_is_blank(hl, p);
    size_t li = li_ + 1;
    int indent = 0;
    if (incr) indent = parent >= 0 ? parent + incr : incr;
    std::string out, leading_break, trailing_breaks;
    // leading breaks; the first non-empty line fixes the indentation
    int max_indent = 0;
    for (;;) {
      if (li >= L_.size()) break;
      const Line& ln = L_[li];
      if (ln.len > 0 && ln.indent == ln.len) throw Unsupported();  // whitespace-only line
      if (ln.len == 0) {
        if (!ln.has_break) break;  // end of input
        trailing_breaks.push_back('\n');
        li++;
        continue;
      }
      if (!indent && ln.indent > max_indent) max_indent = ln.indent;
      break;
    }
    if (!indent) {
      indent = max_indent;
      if (indent < parent + 1) indent = parent + 1;
      if (indent < 1) indent = 1;
    }
    bool leading_blank = false;
    bool ended_at_eof = false;
    while (li < L_.size()) {
      const Line& ln = L_[li];
      if (ln.len == 0 || ln.indent < indent) break;
      const bool trailing_blank = ln.s[indent] == ' ';
      if (!literal && !leading_break.empty() && leading_break[0] == '\n' && !leading_blank && !trailing_blank) {
        if (trailing_breaks.empty()) out.push_back(' ');
        leading_break.clear();
      } else {
        out += leading_break;
        leading_break.clear();
      }
      out += trailing_breaks;
      trailing_breaks.clear();
      leading_blank = trailing_blank;
      out.append(ln.s + indent, (size_t)(ln.len - indent));
      li++;
      if (!ln.has_break) {
        ended_at_eof = true;
        break;
      }
      leading_break = "\n";
      // breaks after the line
      while (li < L_.size()) {
        const Line& b = L_[li];
        if (b.len > 0 && b.indent == b.len) throw Unsupported();
        if (b.len != 0) break;
        if (!b.has_break) break;
        trailing_breaks.push_back('\n');
        li++;
      }
    }
    (void)ended_at_eof;
    if (chomp != -1) out += leading_break;
    if (chomp == 1) out += trailing_breaks;
    li_ = li;
    return str(out.data(), out.size());
  }

  // ---- flow collections (one line) ------------------------------------------
  PyObject* flow(const Line& ln, int pos, int& end) {
    DepthGuard guard(depth_);
    const bool is_seq = ln.s[pos] == '[';
    const char close = is_seq ? ']' : '}';
    Ref coll(is_seq ? PyList_New(0) : PyDict_New());
    std::unordered_set<std::string> seen;
    int p = pos + 1;
    while (p < ln.len && ln.s[p] == ' ') p++;
    if (p < ln.len && ln.s[p] == close) {
      end = p + 1;
      return coll.release();
    }
    for (;;) {
      while (p < ln.len && ln.s[p] == ' ') p++;
      if (p >= ln.len) throw Unsupported();  // multi-line flow
      Ref key;
      if (!is_seq) {
        const int kstart = p;
        key = Ref(flow_scalar(ln, p, p, true));
        if (p - kstart > kMaxSimpleKey) throw Unsupported();
        if (PyObject_Hash(key.get()) == -1) throw PyErrorSet();
        check_unique(coll.get(), key.get(), seen, key_value(key.get(), ln.s + kstart, (size_t)(p - kstart)));
        while (p < ln.len && ln.s[p] == ' ') p++;
        if (!(p < ln.len && ln.s[p] == ':' && p + 1 < ln.len && ln.s[p + 1] == ' ')) throw Unsupported();
        p += 2;
        while (p < ln.len && ln.s[p] == ' ') p++;
        if (p >= ln.len) throw Unsupported();
      }
      Ref v;
      if (ln.s[p] == '[' || ln.s[p] == '{') {
        int e;
        v = Ref(flow(ln, p, e));
        p = e;
      } else {
        v = Ref(flow_scalar(ln, p, p, false));
      }
      while (p < ln.len && ln.s[p] == ' ') p++;
      if (p >= ln.len) throw Unsupported();
      if (ln.s[p] == ':') throw Unsupported();  // single-pair mapping / adjacent value
      if (is_seq) {
        if (PyList_Append(coll.get(), v.get()) < 0) throw PyErrorSet();
      } else if (PyDict_SetItem(coll.get(), key.get(), v.get()) < 0) {
        throw PyErrorSet();
      }
      if (ln.s[p] == close) {
        end = p + 1;
        return coll.release();
      }
      if (ln.s[p] != ',') throw Unsupported();
      p++;
      while (p < ln.len && ln.s[p] == ' ') p++;
      if (p < ln.len && (ln.s[p] == close || ln.s[p] == ',')) throw Unsupported();  // trailing/empty entry
    }
  }

  // a scalar inside a flow collection; `out` is set past it
  PyObject* flow_scalar(const Line& ln, int pos, int& out, bool is_key) {
    const char c = ln.s[pos];
    if (c == '"' || c == '\'') {
      int e;
      std::string v = quoted(ln, pos, e);
      out = e;
      return str(v.data(), v.size());
    }
    if (c == '[' || c == '{') throw Unsupported();  // collection as a key
    check_plain_start(ln, pos, true);
    int e = pos;
    while (e < ln.len) {
      const char d = ln.s[e];
      if (is_flow_ind(d)) break;
      if (d == '#' && ln.s[e - 1] == ' ') throw Unsupported();
      if (d == ':' && (e + 1 == ln.len || ln.s[e + 1] == ' ' || is_flow_ind(ln.s[e + 1]))) {
        if (!is_key) throw Unsupported();
        break;
      }
      e++;
    }
    int t = e;
    while (t > pos && ln.s[t - 1] == ' ') t--;
    if (t == pos) throw Unsupported();
    out = e;
    return plain(ln.s + pos, (size_t)(t - pos));
  }
};

}  // namespace m2kyamlp

// Decode `text` (str).  mode: 0 go-yaml v3 typed, 1 go-yaml v2 typed, 2 raw.
// multi: a list of every document, else the single document (None when empty).
// Returns a new reference to `unsupported` when the input is outside the subset
// (or has more than one document in single mode); NULL with an exception set on
// a Python error.
extern "C" PyObject* m2k_yaml_load(PyObject* text, int mode, int multi, PyObject* resolve_number,
                                   PyObject* unsupported) {
  Py_ssize_t n = 0;
  const char* s = PyUnicode_AsUTF8AndSize(text, &n);
  if (!s) {
    PyErr_Clear();
    Py_INCREF(unsupported);
    return unsupported;
  }
  try {
    m2kyamlp::Parser parser(s, (size_t)n, mode, resolve_number);
    std::vector<m2kyamlp::Ref> docs = parser.stream();
    if (!multi) {
      if (docs.size() > 1) {
        Py_INCREF(unsupported);
        return unsupported;
      }
      if (docs.empty()) {
        Py_INCREF(Py_None);
        return Py_None;
      }
      return docs[0].release();
    }
    PyObject* lst = PyList_New((Py_ssize_t)docs.size());
    if (!lst) return nullptr;
    for (size_t i = 0; i < docs.size(); i++) PyList_SET_ITEM(lst, (Py_ssize_t)i, docs[i].release());
    return lst;
  } catch (const m2kyamlp::Unsupported&) {
    Py_INCREF(unsupported);
    return unsupported;
  } catch (const m2kyamlp::TooDeep&) {
    PyErr_Format(PyExc_ValueError, "yaml: exceeded max depth of %d", m2kyamlp::kMaxDepth);
    return nullptr;
  } catch (const m2kyamlp::PyErrorSet&) {
    return nullptr;
  } catch (const std::bad_alloc&) {
    PyErr_NoMemory();
    return nullptr;
  }
}
