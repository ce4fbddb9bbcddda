// go-yaml v3 compatible block emitter (the hot half of every `translate`:
// each manifest, plan, QA cache and values.yaml goes through it).
//
// Semantics are exactly those of move2kube_amd/utils/yamlio.py::_Emitter (the
// executable specification, itself a re-implementation of libyaml's
// yaml_emitter_analyze_scalar / select_scalar_style as driven by go-yaml v3
// `Encoder.SetIndent(2)`, reference internal/common/utils.go:159-177 and
// internal/transformer/transformer.go:162-204).  This file walks the Python
// object tree with the raw CPython API and writes UTF-8 straight into one
// buffer.  ASCII strings, ints, bools, None, dicts, lists and tuples are
// handled natively; the rare rest (floats, bytes, non-ASCII strings, str/int
// subclasses, non-string map keys, and the numeric-looking-string resolution
// check) is delegated to the Python helpers passed in `helpers`, so the two
// implementations can never drift on those corner cases.

#include <Python.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace m2kyaml {

enum Style { PLAIN = 0, SINGLE = 1, DOUBLE = 2, LITERAL = 3 };

struct Ctx {
  bool sort_maps;
  PyObject* gomap;     // GoMap type
  PyObject* scalar_fn;  // (value, indent, key) -> [lines]
  PyObject* style_fn;   // (str, key) -> Style
  PyObject* sort_fn;    // (keys) -> sorted keys
  std::string out;
};

static inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
static inline bool is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
static inline bool is_break(char c) { return c == '\r' || c == '\n'; }
static inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
static inline bool is_printable(unsigned char c) { return c == 0x0A || (c >= 0x20 && c <= 0x7E); }

static bool eq(const char* s, size_t n, const char* lit) {
  size_t m = std::strlen(lit);
  return n == m && std::memcmp(s, lit, n) == 0;
}

static bool in_list(const char* s, size_t n, const char* const* lits) {
  for (; *lits; ++lits)
    if (eq(s, n, *lits)) return true;
  return false;
}

static const char* const kNulls[] = {"~", "null", "Null", "NULL", nullptr};
static const char* const kBools[] = {"true", "True", "TRUE", "false", "False", "FALSE", nullptr};
static const char* const kOldBools[] = {"y",  "Y",  "yes", "Yes", "YES", "on",  "On",  "ON",
                                        "n",  "N",  "no",  "No",  "NO",  "off", "Off", "OFF", nullptr};

// libyaml scalar analysis restricted to ASCII input.
struct Analysis {
  bool multiline, block_plain, single_ok, block_ok;
};

static Analysis analyze(const char* s, size_t n) {
  if (n == 0) return {false, true, true, false};
  bool block_ind = false, flow_ind = false, line_breaks = false, special = false, tabs = false;
  bool leading_space = false, leading_break = false, trailing_space = false, trailing_break = false;
  bool break_space = false, space_break = false, prev_space = false, prev_break = false;
  if (n >= 3 && (std::memcmp(s, "---", 3) == 0 || std::memcmp(s, "...", 3) == 0)) block_ind = flow_ind = true;
  bool preceded_by_ws = true;
  for (size_t i = 0; i < n; ++i) {
    char ch = s[i];
    bool followed_by_ws = i + 1 >= n || is_ws(s[i + 1]);
    if (i == 0) {
      switch (ch) {
        case '#': case ',': case '[': case ']': case '{': case '}': case '&': case '*': case '!':
        case '|': case '>': case '\'': case '"': case '%': case '@': case '`':
          flow_ind = block_ind = true;
          break;
        case '?': case ':':
          flow_ind = true;
          if (followed_by_ws) block_ind = true;
          break;
        case '-':
          if (followed_by_ws) flow_ind = block_ind = true;
          break;
        default:
          break;
      }
    } else {
      switch (ch) {
        case ',': case '?': case '[': case ']': case '{': case '}':
          flow_ind = true;
          break;
        case ':':
          flow_ind = true;
          if (followed_by_ws) block_ind = true;
          break;
        case '#':
          if (preceded_by_ws) flow_ind = block_ind = true;
          break;
        default:
          break;
      }
    }
    if (ch == '\t')
      tabs = true;
    else if (!is_printable(static_cast<unsigned char>(ch)))
      special = true;
    if (ch == ' ') {
      if (i == 0) leading_space = true;
      if (i == n - 1) trailing_space = true;
      if (prev_break) break_space = true;
      prev_space = true;
      prev_break = false;
    } else if (is_break(ch)) {
      line_breaks = true;
      if (i == 0) leading_break = true;
      if (i == n - 1) trailing_break = true;
      if (prev_space) space_break = true;
      prev_space = false;
      prev_break = true;
    } else {
      prev_space = prev_break = false;
    }
    preceded_by_ws = is_ws(ch) || ch == '\0';
  }
  bool block_plain = true, single_ok = true, block_ok = true;
  if (leading_space || leading_break || trailing_space || trailing_break) block_plain = false;
  if (trailing_space) block_ok = false;
  if (break_space) block_plain = single_ok = false;
  if (space_break || tabs || special) block_plain = single_ok = false;
  if (space_break || special) block_ok = false;
  if (line_breaks) block_plain = false;
  if (block_ind) block_plain = false;
  return {line_breaks, block_plain, single_ok, block_ok};
}

// A null, a bool (YAML 1.1 words included) or the merge key: never plain.
static bool reserved_word(const char* s, size_t n) {
  switch (s[0]) {  // every such word starts with one of these
    case '~': case 'n': case 'N': case 't': case 'T': case 'f': case 'F':
    case 'y': case 'Y': case 'o': case 'O': case '<':
      break;
    default:
      return false;
  }
  return in_list(s, n, kNulls) || in_list(s, n, kBools) || in_list(s, n, kOldBools) || eq(s, n, "<<");
}

// Style for an ASCII string; -1 with a Python error set on failure.
static int string_style(Ctx& c, PyObject* str, const char* s, size_t n, bool key) {
  bool can_plain;
  if (n > 0 && (is_digit(s[0]) || s[0] == '+' || s[0] == '-' || s[0] == '.')) {
    // number / timestamp / base-60 resolution: ask the Python specification
    PyObject* r = PyObject_CallFunction(c.style_fn, "OO", str, key ? Py_True : Py_False);
    if (!r) return -1;
    long v = PyLong_AsLong(r);
    Py_DECREF(r);
    if (v == -1 && PyErr_Occurred()) return -1;
    return static_cast<int>(v);
  }
  can_plain = n > 0 && !reserved_word(s, n);
  int style;
  if (std::memchr(s, '\n', n))
    style = LITERAL;
  else if (can_plain)
    style = PLAIN;
  else
    style = DOUBLE;
  Analysis a = analyze(s, n);
  if (key && a.multiline) style = DOUBLE;
  if (style == PLAIN) {
    if (!a.block_plain) style = SINGLE;
    if (n == 0 && key) style = SINGLE;
  }
  if (style == SINGLE && !a.single_ok) style = DOUBLE;
  if (style == LITERAL && (!a.block_ok || key)) style = DOUBLE;
  return style;
}

static void put_double_quoted(std::string& o, const char* s, size_t n) {
  static const char hex[] = "0123456789ABCDEF";
  o.push_back('"');
  for (size_t i = 0; i < n; ++i) {
    unsigned char ch = static_cast<unsigned char>(s[i]);
    switch (ch) {
      case 0x00: o += "\\0"; break;
      case 0x07: o += "\\a"; break;
      case 0x08: o += "\\b"; break;
      case '\t': o += "\\t"; break;
      case '\n': o += "\\n"; break;
      case 0x0B: o += "\\v"; break;
      case 0x0C: o += "\\f"; break;
      case '\r': o += "\\r"; break;
      case 0x1B: o += "\\e"; break;
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      default:
        if (is_printable(ch)) {
          o.push_back(static_cast<char>(ch));
        } else {
          o += "\\x";
          o.push_back(hex[ch >> 4]);
          o.push_back(hex[ch & 15]);
        }
    }
  }
  o.push_back('"');
}

static void put_single_quoted(std::string& o, const char* s, size_t n) {
  o.push_back('\'');
  for (size_t i = 0; i < n; ++i) {
    if (s[i] == '\'') o.push_back('\'');
    o.push_back(s[i]);
  }
  o.push_back('\'');
}

// Header line plus content lines, separated (not terminated) by '\n'.
static void put_literal(std::string& o, const char* s, size_t n, int indent) {
  o.push_back('|');
  if (n > 0 && (s[0] == ' ' || is_break(s[0]))) o.push_back('2');
  if (n == 0 || !is_break(s[n - 1]))
    o.push_back('-');
  else if (n == 1 || is_break(s[n - 2]))
    o.push_back('+');
  bool breaks = true;
  bool open = false;  // a content line is being built
  for (size_t i = 0; i < n; ++i) {
    char ch = s[i];
    if (is_break(ch)) {
      if (!open) o.push_back('\n');  // empty line
      open = false;
      breaks = true;
    } else {
      if (breaks) {
        o.push_back('\n');
        o.append(static_cast<size_t>(indent), ' ');
        breaks = false;
        open = true;
      }
      o.push_back(ch);
    }
  }
}

// Python fallback: scalar_fn(v, indent, key) -> list of lines.
static bool scalar_fallback(Ctx& c, PyObject* v, int indent, bool key) {
  PyObject* lines = PyObject_CallFunction(c.scalar_fn, "OiO", v, indent, key ? Py_True : Py_False);
  if (!lines) return false;
  Py_ssize_t n = PyList_Size(lines);
  if (n < 0) {
    Py_DECREF(lines);
    return false;
  }
  Py_ssize_t upto = key ? std::min<Py_ssize_t>(n, 1) : n;
  for (Py_ssize_t i = 0; i < upto; ++i) {
    // surrogatepass: lone surrogates (surrogateescape'd file names) round-trip
    PyObject* b = PyUnicode_AsEncodedString(PyList_GET_ITEM(lines, i), "utf-8", "surrogatepass");
    if (!b) {
      Py_DECREF(lines);
      return false;
    }
    if (i) c.out.push_back('\n');
    c.out.append(PyBytes_AS_STRING(b), static_cast<size_t>(PyBytes_GET_SIZE(b)));
    Py_DECREF(b);
  }
  Py_DECREF(lines);
  return true;
}

static bool put_scalar(Ctx& c, PyObject* v, int indent, bool key) {
  if (v == Py_None) {
    c.out += "null";
    return true;
  }
  if (v == Py_True) {
    c.out += "true";
    return true;
  }
  if (v == Py_False) {
    c.out += "false";
    return true;
  }
  if (PyLong_CheckExact(v)) {
    int overflow = 0;
    long long x = PyLong_AsLongLongAndOverflow(v, &overflow);
    if (!overflow) {
      if (x == -1 && PyErr_Occurred()) return false;
      c.out += std::to_string(x);
      return true;
    }
    return scalar_fallback(c, v, indent, key);
  }
  if (PyUnicode_CheckExact(v) && PyUnicode_IS_ASCII(v)) {
    Py_ssize_t len;
    const char* s = PyUnicode_AsUTF8AndSize(v, &len);
    if (!s) return false;
    size_t n = static_cast<size_t>(len);
    int st = string_style(c, v, s, n, key);
    switch (st) {
      case PLAIN: c.out.append(s, n); return true;
      case SINGLE: put_single_quoted(c.out, s, n); return true;
      case DOUBLE: put_double_quoted(c.out, s, n); return true;
      case LITERAL: put_literal(c.out, s, n, indent); return true;
      default: return false;  // error from style_fn
    }
  }
  return scalar_fallback(c, v, indent, key);
}

// go-yaml v3 sorter.go keyList.Less on ASCII strings (unbounded digit runs,
// like the Python specification).
static int cmp_digit_runs(bool one_a, const char* a, size_t na, bool one_b, const char* b, size_t nb) {
  // value of ("1" if one) + digits, compared numerically
  std::string x = one_a ? "1" : "", y = one_b ? "1" : "";
  x.append(a, na);
  y.append(b, nb);
  size_t i = x.find_first_not_of('0'), j = y.find_first_not_of('0');
  const char* px = i == std::string::npos ? "" : x.c_str() + i;
  const char* py = j == std::string::npos ? "" : y.c_str() + j;
  size_t lx = std::strlen(px), ly = std::strlen(py);
  if (lx != ly) return lx < ly ? -1 : 1;
  int r = std::memcmp(px, py, lx);
  return r < 0 ? -1 : (r > 0 ? 1 : 0);
}

static int go_key_cmp(const char* a, size_t na, const char* b, size_t nb) {
  bool digits = false;
  size_t n = std::min(na, nb);
  for (size_t i = 0; i < n; ++i) {
    if (a[i] == b[i]) {
      digits = is_digit(a[i]);
      continue;
    }
    bool al = is_alpha(a[i]), bl = is_alpha(b[i]);
    if (al && bl) return a[i] < b[i] ? -1 : 1;
    if (al || bl) {
      if (digits) return al ? -1 : 1;
      return bl ? -1 : 1;
    }
    bool one = false;
    if (a[i] == '0' || b[i] == '0') {
      for (size_t j = i; j-- > 0 && is_digit(a[j]);) {
        if (a[j] != '0') {
          one = true;
          break;
        }
      }
    }
    size_t ai = i, bi = i;
    while (ai < na && is_digit(a[ai])) ++ai;
    while (bi < nb && is_digit(b[bi])) ++bi;
    int r = cmp_digit_runs(one, a + i, ai - i, one, b + i, bi - i);
    if (r) return r;
    if (ai != bi) return ai < bi ? -1 : 1;
    return a[i] < b[i] ? -1 : 1;
  }
  return na < nb ? -1 : (na > nb ? 1 : 0);
}

struct Entry {
  PyObject* key;  // borrowed
  PyObject* val;  // borrowed
  const char* s;
  size_t n;
};

// A line's lead-in is `indent` columns: spaces, or - for the first entry of a
// mapping or sequence that is itself a sequence item - spaces followed by
// `marks` "- " pairs (a sequence item's dash(es) on the same line).
static bool emit_value_tail(Ctx& c, PyObject* v, int indent);
static bool emit_map(Ctx& c, PyObject* d, int indent, int first_marks);
static bool emit_seq(Ctx& c, PyObject* seq, int indent, int first_marks);

static inline void put_lead(Ctx& c, int indent, int marks) {
  c.out.append(static_cast<size_t>(indent - 2 * marks), ' ');
  for (int i = 0; i < marks; ++i) c.out += "- ";
}

static inline bool is_seq(PyObject* v) { return PyList_Check(v) || PyTuple_Check(v); }
static inline Py_ssize_t seq_len(PyObject* v) { return PyList_Check(v) ? PyList_GET_SIZE(v) : PyTuple_GET_SIZE(v); }
static inline PyObject* seq_item(PyObject* v, Py_ssize_t i) {
  return PyList_Check(v) ? PyList_GET_ITEM(v, i) : PyTuple_GET_ITEM(v, i);
}

static bool emit_entry(Ctx& c, PyObject* k, PyObject* v, int indent, int marks) {
  put_lead(c, indent, marks);
  if (!put_scalar(c, k, indent, true)) return false;
  c.out.push_back(':');
  return emit_value_tail(c, v, indent);
}

static bool emit_map(Ctx& c, PyObject* d, int indent, int first_marks) {
  int sorted = c.sort_maps;
  if (!sorted) {
    sorted = PyObject_IsInstance(d, c.gomap);
    if (sorted < 0) return false;
  }
  bool plain_dict = PyDict_CheckExact(d) || Py_TYPE(d) == reinterpret_cast<PyTypeObject*>(c.gomap);
  if (!sorted && plain_dict) {
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    bool first = true;
    while (PyDict_Next(d, &pos, &k, &v)) {
      if (!emit_entry(c, k, v, indent, first ? first_marks : 0)) return false;
      first = false;
    }
    return true;
  }
  if (plain_dict) {
    // small maps (nearly all of a manifest's) sort on the stack by insertion
    const size_t size = static_cast<size_t>(PyDict_GET_SIZE(d));
    Entry small[32];
    std::vector<Entry> big;
    Entry* es = small;
    if (size > 32) {
      big.resize(size);
      es = big.data();
    }
    size_t n = 0;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    bool native_keys = true;
    while (PyDict_Next(d, &pos, &k, &v)) {
      if (!PyUnicode_CheckExact(k) || !PyUnicode_IS_ASCII(k)) {
        native_keys = false;
        break;
      }
      // compact ASCII: the UTF-8 form is the string's own data
      es[n++] = {k, v, static_cast<const char*>(PyUnicode_DATA(k)), static_cast<size_t>(PyUnicode_GET_LENGTH(k))};
    }
    if (native_keys) {
      auto less = [](const Entry& x, const Entry& y) { return go_key_cmp(x.s, x.n, y.s, y.n) < 0; };
      if (n > 32) {
        std::stable_sort(es, es + n, less);
      } else {
        for (size_t i = 1; i < n; ++i) {   // stable: an entry moves only past strictly greater ones
          Entry e = es[i];
          size_t j = i;
          for (; j > 0 && less(e, es[j - 1]); --j) es[j] = es[j - 1];
          es[j] = e;
        }
      }
      for (size_t i = 0; i < n; ++i)
        if (!emit_entry(c, es[i].key, es[i].val, indent, i == 0 ? first_marks : 0)) return false;
      return true;
    }
  }
  // generic mapping (dict subclass) or non-string keys: Python key order
  PyObject* keys = PyMapping_Keys(d);
  if (!keys) return false;
  if (sorted) {
    PyObject* s = PyObject_CallFunctionObjArgs(c.sort_fn, keys, nullptr);
    Py_DECREF(keys);
    if (!s) return false;
    keys = s;
  }
  PyObject* list = PySequence_Fast(keys, "keys");
  Py_DECREF(keys);
  if (!list) return false;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(list);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* k = PySequence_Fast_GET_ITEM(list, i);
    PyObject* v = PyObject_GetItem(d, k);
    if (!v) {
      Py_DECREF(list);
      return false;
    }
    bool ok = emit_entry(c, k, v, indent, i == 0 ? first_marks : 0);
    Py_DECREF(v);
    if (!ok) {
      Py_DECREF(list);
      return false;
    }
  }
  Py_DECREF(list);
  return true;
}

static bool emit_seq(Ctx& c, PyObject* seq, int indent, int first_marks) {
  Py_ssize_t n = seq_len(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* item = seq_item(seq, i);
    const int marks = i == 0 ? first_marks : 0;   // this item's lead-in, then its own "- "
    if (PyDict_Check(item)) {
      if (PyDict_GET_SIZE(item) > 0) {
        if (!emit_map(c, item, indent + 2, marks + 1)) return false;
      } else {
        put_lead(c, indent, marks);
        c.out += "- {}\n";
      }
    } else if (is_seq(item)) {
      if (seq_len(item) > 0) {
        if (!emit_seq(c, item, indent + 2, marks + 1)) return false;
      } else {
        put_lead(c, indent, marks);
        c.out += "- []\n";
      }
    } else {
      put_lead(c, indent, marks);
      c.out += "- ";
      if (!put_scalar(c, item, indent + 2, false)) return false;
      c.out.push_back('\n');
    }
  }
  return true;
}

// After "<prefix>key:" - the value part of a mapping entry.
static bool emit_value_tail(Ctx& c, PyObject* v, int indent) {
  if (PyDict_Check(v)) {
    if (PyDict_GET_SIZE(v) == 0) {
      c.out += " {}\n";
      return true;
    }
    c.out.push_back('\n');
    return emit_map(c, v, indent + 2, 0);
  }
  if (is_seq(v)) {
    if (seq_len(v) == 0) {
      c.out += " []\n";
      return true;
    }
    c.out.push_back('\n');
    return emit_seq(c, v, indent + 2, 0);
  }
  c.out.push_back(' ');
  if (!put_scalar(c, v, indent + 2, false)) return false;
  c.out.push_back('\n');
  return true;
}

}  // namespace m2kyaml

// dump(data, sort_maps, gomap_type, scalar_fn, style_fn, sort_fn) -> str
extern "C" PyObject* m2k_yaml_dump(PyObject* data, int sort_maps, PyObject* gomap, PyObject* scalar_fn,
                                   PyObject* style_fn, PyObject* sort_fn) {
  using namespace m2kyaml;
  Ctx c{sort_maps != 0, gomap, scalar_fn, style_fn, sort_fn, std::string()};
  c.out.reserve(4096);
  bool ok;
  if (PyDict_Check(data)) {
    if (PyDict_GET_SIZE(data) == 0) {
      c.out += "{}\n";
      ok = true;
    } else {
      ok = emit_map(c, data, 0, 0);
    }
  } else if (is_seq(data)) {
    if (seq_len(data) == 0) {
      c.out += "[]\n";
      ok = true;
    } else {
      ok = emit_seq(c, data, 0, 0);
    }
  } else {
    ok = put_scalar(c, data, 2, false);
    if (ok) c.out.push_back('\n');
  }
  if (!ok) return nullptr;
  return PyUnicode_DecodeUTF8(c.out.data(), static_cast<Py_ssize_t>(c.out.size()), "surrogatepass");
}
