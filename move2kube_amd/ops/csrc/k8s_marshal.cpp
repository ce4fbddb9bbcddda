// Go encoding/json struct-tag marshalling of the typed Kubernetes objects:
// the native twin of move2kube_amd/k8s/schema.py::_marshal_struct, run on
// every manifest `translate` writes (reference
// internal/transformer/transformer.go:162-204 marshals each object through
// its Go struct before the YAML encoder).
//
// schema.py stays the executable specification.  At first use it hands its
// struct table (name -> its field DSL string, or [(json name, field type,
// omitempty)]) to `schema_init`, which parses and compiles every field once; `schema_marshal(obj,
// type)` then walks the JSON-shaped Python tree with the raw CPython API and
// returns the same dict tree the Python code builds (same keys, same key
// order, the same shared per-type empty-struct dicts).  Anything outside the
// plain shapes - a non-dict where a struct is expected, a non-dict map, the
// bytes / RawExtension field types - is handed back to the Python
// implementation (`fallback(value, type)`), so both paths raise the same
// errors on malformed objects.

#include <Python.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace m2kschema {

enum Kind { K_IDENT, K_PTR, K_SLICE, K_MAP_PLAIN, K_MAP_OF, K_STR, K_BOOL, K_TIME, K_STRUCT, K_FALLBACK };
enum Empty { E_NEVER, E_STR, E_INT, E_BOOL, E_LEN, E_ANY };
enum Absent { A_SKIP, A_NONE, A_EMPTY_STRUCT, A_ZERO_STR, A_ZERO_INT, A_ZERO_BOOL };

struct Type {
  Kind kind;
  int inner;   // element / pointee type (index into types)
  int strct;   // struct index for K_STRUCT
  PyObject* name;  // type string (for the fallback call)
};

struct Field {
  PyObject* jname;
  int type;
  bool omit;
  bool inline_;
  Empty empty;
  Absent absent;
};

struct Struct {
  std::string name;
  PyObject* spec = nullptr;   // its fields as schema.py handed them (compiled on first use)
  bool compiled = false;
  std::vector<Field> fields;
  PyObject* keyed = nullptr;  // json name -> field index (PyLong)
  std::vector<int> inlines;   // struct indices
  PyObject* base = nullptr;   // fields an absent key still produces
  PyObject* empty = nullptr;  // the marshalled empty struct (shared)
  bool building = false;
};

struct Schema {
  std::vector<Type> types;
  std::unordered_map<std::string, int> type_index;
  std::vector<Struct> structs;
  std::unordered_map<std::string, int> struct_index;
  PyObject* fallback = nullptr;  // (value, type) -> marshalled value
  PyObject* zero = nullptr;      // 0
  PyObject* empty_str = nullptr;  // ""
  bool ready = false;             // set once every struct compiled
};

static Schema* g = nullptr;

// Drop a schema whose compilation failed part-way, so that no marshal call can
// see a struct without its field table and a later init starts afresh.
static void discard_schema() {
  if (g == nullptr) return;
  for (Type& t : g->types) Py_XDECREF(t.name);
  for (Struct& s : g->structs) {
    for (Field& f : s.fields) Py_XDECREF(f.jname);
    Py_XDECREF(s.spec);
    Py_XDECREF(s.keyed);
    Py_XDECREF(s.base);
    Py_XDECREF(s.empty);
  }
  Py_XDECREF(g->fallback);
  Py_XDECREF(g->zero);
  Py_XDECREF(g->empty_str);
  delete g;
  g = nullptr;
}

static int compile_type(const std::string& t);

static int add_type(const std::string& t, Kind k, int inner, int strct) {
  Type ty{k, inner, strct, PyUnicode_FromStringAndSize(t.data(), (Py_ssize_t)t.size())};
  g->types.push_back(ty);
  int ix = (int)g->types.size() - 1;
  g->type_index[t] = ix;
  return ix;
}

static int compile_type(const std::string& t) {
  auto it = g->type_index.find(t);
  if (it != g->type_index.end()) return it->second;
  if (t.rfind("*", 0) == 0) return add_type(t, K_PTR, compile_type(t.substr(1)), -1);
  if (t.rfind("[]", 0) == 0) return add_type(t, K_SLICE, compile_type(t.substr(2)), -1);
  if (t == "map") return add_type(t, K_MAP_PLAIN, -1, -1);
  if (t.rfind("map:", 0) == 0) return add_type(t, K_MAP_OF, compile_type(t.substr(4)), -1);
  if (t == "bytes" || t == "RawExtension") return add_type(t, K_FALLBACK, -1, -1);
  if (t == "Time") return add_type(t, K_TIME, -1, -1);
  if (t == "string" || t == "Quantity" || t == "ArrayOrString") return add_type(t, K_STR, -1, -1);
  if (t == "bool") return add_type(t, K_BOOL, -1, -1);
  auto s = g->struct_index.find(t);
  if (s != g->struct_index.end()) return add_type(t, K_STRUCT, -1, s->second);
  return add_type(t, K_IDENT, -1, -1);  // int, IntOrString, any, unknown
}

static Empty empty_kind(const std::string& t) {
  if (t.rfind("*", 0) == 0) return E_NEVER;
  if (t == "string") return E_STR;
  if (t == "int") return E_INT;
  if (t == "bool") return E_BOOL;
  if (t.rfind("[]", 0) == 0 || t.rfind("map", 0) == 0 || t == "bytes") return E_LEN;
  if (t == "any") return E_ANY;
  return E_NEVER;
}

static Absent absent_kind(const std::string& t, bool omit) {
  if (g->struct_index.count(t)) return A_EMPTY_STRUCT;
  if (t == "Time") return A_NONE;
  if (omit) return A_SKIP;
  if (t.rfind("*", 0) == 0 || t.rfind("[]", 0) == 0 || t.rfind("map", 0) == 0 || t == "any" || t == "bytes")
    return A_NONE;
  if (t == "string" || t == "ArrayOrString") return A_ZERO_STR;
  if (t == "int" || t == "IntOrString") return A_ZERO_INT;
  if (t == "bool") return A_ZERO_BOOL;
  return A_NONE;
}

static PyObject* marshal_value(PyObject* v, int type);
static PyObject* marshal_struct(PyObject* d, int strct);

// the marshalled empty struct of `strct` (borrowed; cached)
static PyObject* empty_struct(int strct);

// compiles a struct's field table on its first use (false + exception on error)
static bool ensure(int strct);

static PyObject* base_of(int strct) {
  Struct& s = g->structs[strct];
  if (s.base) return s.base;
  if (!ensure(strct)) return nullptr;
  PyObject* base = PyDict_New();
  if (!base) return nullptr;
  for (const Field& f : s.fields) {
    if (f.inline_ || f.absent == A_SKIP) continue;
    PyObject* v = nullptr;
    switch (f.absent) {
      case A_EMPTY_STRUCT: {
        PyObject* e = empty_struct(g->types[f.type].strct);
        if (!e) { Py_DECREF(base); return nullptr; }
        Py_INCREF(e);
        v = e;
        break;
      }
      case A_ZERO_STR: Py_INCREF(g->empty_str); v = g->empty_str; break;
      case A_ZERO_INT: Py_INCREF(g->zero); v = g->zero; break;
      case A_ZERO_BOOL: Py_INCREF(Py_False); v = Py_False; break;
      default: Py_INCREF(Py_None); v = Py_None; break;
    }
    int rc = PyDict_SetItem(base, f.jname, v);
    Py_DECREF(v);
    if (rc < 0) { Py_DECREF(base); return nullptr; }
  }
  s.base = base;
  return base;
}

static PyObject* empty_struct(int strct) {
  Struct& s = g->structs[strct];
  if (s.empty) return s.empty;
  if (s.building) {
    PyErr_SetString(PyExc_RecursionError, "recursive struct type");
    return nullptr;
  }
  s.building = true;
  PyObject* base = base_of(strct);
  PyObject* out = base ? PyDict_Copy(base) : nullptr;
  if (out) {
    for (int in : s.inlines) {
      PyObject* e = empty_struct(in);
      if (!e || PyDict_Update(out, e) < 0) { Py_CLEAR(out); break; }
    }
  }
  s.building = false;
  s.empty = out;
  return out;
}

static int is_empty(PyObject* v, Empty e) {
  switch (e) {
    case E_NEVER: return 0;
    case E_STR: return PyObject_RichCompareBool(v, g->empty_str, Py_EQ);
    case E_INT: return PyObject_RichCompareBool(v, g->zero, Py_EQ);
    case E_BOOL: return v == Py_False;
    case E_LEN: {
      Py_ssize_t n = PyObject_Length(v);
      return n < 0 ? -1 : n == 0;
    }
    case E_ANY: {
      if (PyDict_Check(v) || PyList_Check(v) || PyUnicode_Check(v)) {
        Py_ssize_t n = PyObject_Length(v);
        if (n < 0) return -1;
        if (n == 0) return 1;
      }
      if (v == Py_False) return 1;
      return PyObject_RichCompareBool(v, g->zero, Py_EQ);
    }
  }
  return 0;
}

static PyObject* fallback(PyObject* v, int type) {
  return PyObject_CallFunctionObjArgs(g->fallback, v, g->types[type].name, nullptr);
}

static PyObject* marshal_fields(PyObject* d, int strct) {
  Struct& s = g->structs[strct];
  PyObject* base = base_of(strct);  // compiles the struct on first use
  if (!base) return nullptr;
  PyObject* out = PyDict_Copy(base);
  if (!out) return nullptr;
  for (int in : s.inlines) {
    PyObject* sub = marshal_struct(d, in);
    if (!sub) { Py_DECREF(out); return nullptr; }
    int rc = PyDict_Update(out, sub);
    Py_DECREF(sub);
    if (rc < 0) { Py_DECREF(out); return nullptr; }
  }
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(d, &pos, &k, &v)) {
    PyObject* fi = PyDict_GetItemWithError(s.keyed, k);
    if (!fi) {
      if (PyErr_Occurred()) { Py_DECREF(out); return nullptr; }
      continue;
    }
    if (v == Py_None) continue;
    const Field& f = s.fields[PyLong_AsSsize_t(fi)];
    if (f.omit) {
      int e = is_empty(v, f.empty);
      if (e < 0) { Py_DECREF(out); return nullptr; }
      if (e) {
        if (PyDict_DelItem(out, k) < 0) {
          if (!PyErr_ExceptionMatches(PyExc_KeyError)) { Py_DECREF(out); return nullptr; }
          PyErr_Clear();
        }
        continue;
      }
    }
    PyObject* mv = marshal_value(v, f.type);
    if (!mv) { Py_DECREF(out); return nullptr; }
    int rc = PyDict_SetItem(out, k, mv);
    Py_DECREF(mv);
    if (rc < 0) { Py_DECREF(out); return nullptr; }
  }
  return out;
}

static PyObject* marshal_struct(PyObject* d, int strct) {
  int truth = PyObject_IsTrue(d);
  if (truth < 0) return nullptr;
  if (!truth) {
    PyObject* e = empty_struct(strct);
    Py_XINCREF(e);
    return e;
  }
  if (!PyDict_Check(d)) {  // not a JSON object: the Python code decides (and raises)
    PyObject* name = PyUnicode_FromString(g->structs[strct].name.c_str());
    if (!name) return nullptr;
    PyObject* r = PyObject_CallFunctionObjArgs(g->fallback, d, name, nullptr);
    Py_DECREF(name);
    return r;
  }
  return marshal_fields(d, strct);
}

static PyObject* marshal_value(PyObject* v, int type) {
  const Type t = g->types[type];  // a copy: compiling a struct on first use may grow g->types
  switch (t.kind) {
    case K_IDENT:
      Py_INCREF(v);
      return v;
    case K_PTR:
      if (v == Py_None) Py_RETURN_NONE;
      return marshal_value(v, t.inner);
    case K_SLICE: {
      if (v == Py_None) Py_RETURN_NONE;
      PyObject* it = PyObject_GetIter(v);
      if (!it) return nullptr;
      PyObject* out = PyList_New(0);
      if (!out) { Py_DECREF(it); return nullptr; }
      PyObject* x;
      while ((x = PyIter_Next(it))) {
        PyObject* mx = marshal_value(x, t.inner);
        Py_DECREF(x);
        if (!mx || PyList_Append(out, mx) < 0) {
          Py_XDECREF(mx);
          Py_DECREF(it);
          Py_DECREF(out);
          return nullptr;
        }
        Py_DECREF(mx);
      }
      Py_DECREF(it);
      if (PyErr_Occurred()) { Py_DECREF(out); return nullptr; }
      return out;
    }
    case K_MAP_PLAIN: {
      if (v == Py_None) Py_RETURN_NONE;
      if (PyDict_Check(v)) {
        PyObject* out = PyDict_New();
        if (out && PyDict_Update(out, v) < 0) Py_CLEAR(out);
        return out;
      }
      return PyObject_CallOneArg((PyObject*)&PyDict_Type, v);
    }
    case K_MAP_OF: {
      if (v == Py_None) Py_RETURN_NONE;
      if (!PyDict_Check(v)) return fallback(v, type);
      PyObject* out = PyDict_New();
      if (!out) return nullptr;
      Py_ssize_t pos = 0;
      PyObject *k, *x;
      while (PyDict_Next(v, &pos, &k, &x)) {
        PyObject* mx = marshal_value(x, t.inner);
        if (!mx || PyDict_SetItem(out, k, mx) < 0) {
          Py_XDECREF(mx);
          Py_DECREF(out);
          return nullptr;
        }
        Py_DECREF(mx);
      }
      return out;
    }
    case K_STR:
      if (PyUnicode_Check(v)) { Py_INCREF(v); return v; }
      if (v == Py_None) { Py_INCREF(g->empty_str); return g->empty_str; }
      Py_INCREF(v);
      return v;
    case K_BOOL: {
      int b = PyObject_IsTrue(v);
      if (b < 0) return nullptr;
      return PyBool_FromLong(b);
    }
    case K_TIME: {
      int b = PyObject_IsTrue(v);
      if (b < 0) return nullptr;
      if (!b) Py_RETURN_NONE;
      Py_INCREF(v);
      return v;
    }
    case K_STRUCT: {
      int b = PyObject_IsTrue(v);
      if (b < 0) return nullptr;
      if (!b) {
        PyObject* e = empty_struct(t.strct);
        Py_XINCREF(e);
        return e;
      }
      return marshal_struct(v, t.strct);
    }
    case K_FALLBACK:
      return fallback(v, type);
  }
  Py_INCREF(v);
  return v;
}

}  // namespace m2kschema

namespace m2kschema {

struct FieldSpec {
  std::string jname, ftype;
  bool omit;
};

static bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// One struct's fields, from either form schema.py can hand over: its field
// DSL string ("jsonName:type[,o] ...", split on whitespace as str.split()
// does for ASCII) or a sequence of (json name, field type, omitempty).
static bool field_specs(PyObject* fields, std::vector<FieldSpec>& out) {
  if (PyUnicode_Check(fields)) {
    Py_ssize_t n = 0;
    const char* c = PyUnicode_AsUTF8AndSize(fields, &n);
    if (!c) return false;
    std::string src(c, (size_t)n);
    size_t i = 0;
    while (i < src.size()) {
      while (i < src.size() && is_space(src[i])) ++i;
      size_t j = i;
      while (j < src.size() && !is_space(src[j])) ++j;
      if (j == i) break;
      std::string item = src.substr(i, j - i);
      i = j;
      FieldSpec f;
      f.omit = item.size() >= 2 && item.compare(item.size() - 2, 2, ",o") == 0;
      if (f.omit) item.resize(item.size() - 2);
      size_t colon = item.find(':');
      if (colon == std::string::npos) {
        PyErr_Format(PyExc_ValueError, "field %s has no type", item.c_str());
        return false;
      }
      f.jname = item.substr(0, colon);
      f.ftype = item.substr(colon + 1);
      out.push_back(std::move(f));
    }
    return true;
  }
  PyObject* seq = PySequence_Fast(fields, "fields must be a sequence or a field string");
  if (!seq) return false;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject *jn, *ft, *om;
    const char *jc = nullptr, *fc = nullptr;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(seq, i), "UUO", &jn, &ft, &om) ||
        (jc = PyUnicode_AsUTF8(jn)) == nullptr || (fc = PyUnicode_AsUTF8(ft)) == nullptr) {
      Py_DECREF(seq);
      return false;
    }
    int truth = PyObject_IsTrue(om);
    if (truth < 0) {
      Py_DECREF(seq);
      return false;
    }
    out.push_back(FieldSpec{jc, fc, truth == 1});
  }
  Py_DECREF(seq);
  return true;
}

static bool check_inline(const std::string& ftype) {
  if (g->struct_index.count(ftype)) return true;
  PyErr_Format(PyExc_ValueError, "inline type %s is not a struct", ftype.c_str());
  return false;
}

// What compiling ``fields`` would refuse, without compiling it.
static bool check_spec(PyObject* fields) {
  if (PyUnicode_Check(fields)) {
    Py_ssize_t n = 0;
    const char* c = PyUnicode_AsUTF8AndSize(fields, &n);
    if (!c) return false;
    size_t i = 0, len = (size_t)n;
    while (i < len) {
      while (i < len && is_space(c[i])) ++i;
      size_t j = i;
      while (j < len && !is_space(c[j])) ++j;
      if (j == i) break;
      std::string item(c + i, j - i);
      i = j;
      if (item.size() >= 2 && item.compare(item.size() - 2, 2, ",o") == 0) item.resize(item.size() - 2);
      size_t colon = item.find(':');
      if (colon == std::string::npos) {
        PyErr_Format(PyExc_ValueError, "field %s has no type", item.c_str());
        return false;
      }
      if (item.compare(0, colon, "inline") == 0 && colon == 6 && !check_inline(item.substr(colon + 1))) return false;
    }
    return true;
  }
  std::vector<FieldSpec> specs;
  if (!field_specs(fields, specs)) return false;
  for (const FieldSpec& f : specs)
    if (f.jname == "inline" && !check_inline(f.ftype)) return false;
  return true;
}

static bool ensure(int strct) {
  Struct& s = g->structs[strct];
  if (s.compiled) return true;
  // a compile that fails part-way leaves the struct as it was: uncompiled
  auto fail = [&s]() {
    for (Field& f : s.fields) Py_XDECREF(f.jname);
    s.fields.clear();
    s.inlines.clear();
    if (s.keyed) PyDict_Clear(s.keyed);
    return false;
  };
  std::vector<FieldSpec> specs;
  s.keyed = s.keyed ? s.keyed : PyDict_New();
  if (!s.keyed || !field_specs(s.spec, specs)) return fail();
  for (FieldSpec& spec : specs) {
    const std::string &jname = spec.jname, &ftype = spec.ftype;
    const bool omit = spec.omit;
    PyObject* jn = PyUnicode_FromStringAndSize(jname.data(), (Py_ssize_t)jname.size());
    if (!jn) return fail();
    Field f;
    f.jname = jn;  // owns the reference
    f.omit = omit;
    f.inline_ = jname == "inline";
    f.type = compile_type(ftype);
    f.empty = omit ? empty_kind(ftype) : E_NEVER;
    f.absent = f.inline_ ? A_SKIP : absent_kind(ftype, omit);
    if (f.inline_) {
      auto si = g->struct_index.find(ftype);
      if (si == g->struct_index.end()) {  // check_spec refused this at init
        Py_DECREF(jn);
        PyErr_Format(PyExc_ValueError, "inline type %s is not a struct", ftype.c_str());
        return fail();
      }
      s.inlines.push_back(si->second);
    } else {
      PyObject* idx = PyLong_FromSsize_t((Py_ssize_t)s.fields.size());
      int rc = idx ? PyDict_SetItem(s.keyed, jn, idx) : -1;
      Py_XDECREF(idx);
      if (rc < 0) {
        Py_DECREF(jn);
        return fail();
      }
    }
    s.fields.push_back(f);
  }
  s.compiled = true;
  return true;
}

}  // namespace m2kschema

using namespace m2kschema;

// schema_init(structs: {name: "field DSL" | [(jname, ftype, omit)]}, fallback) -> None
extern "C" PyObject* m2k_schema_init(PyObject* structs, PyObject* fb) {
  if (!PyDict_Check(structs)) {
    PyErr_SetString(PyExc_TypeError, "structs must be a dict");
    return nullptr;
  }
  if (g != nullptr && g->ready) Py_RETURN_NONE;  // already compiled (the table never changes)
  discard_schema();
  g = new Schema();
  g->zero = PyLong_FromLong(0);
  g->empty_str = PyUnicode_FromString("");
  if (g->zero == nullptr || g->empty_str == nullptr) {
    discard_schema();
    return nullptr;
  }
  Py_INCREF(fb);
  g->fallback = fb;
  Py_ssize_t pos = 0;
  PyObject *name, *fields;
  while (PyDict_Next(structs, &pos, &name, &fields)) {
    const char* nm = PyUnicode_Check(name) ? PyUnicode_AsUTF8(name) : nullptr;
    if (nm == nullptr) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "struct names must be str");
      discard_schema();
      return nullptr;
    }
    Struct s;
    s.name = nm;
    g->struct_index[s.name] = (int)g->structs.size();
    g->structs.push_back(std::move(s));
  }
  // keep each struct's spec and check what a compile would refuse: a field
  // without a type, an inline field naming no struct.  The field tables are
  // compiled per struct on first use (ensure): a run marshals a few dozen of
  // the table's structs.
  pos = 0;
  int ix = 0;
  while (PyDict_Next(structs, &pos, &name, &fields)) {
    Struct& s = g->structs[ix++];
    Py_INCREF(fields);
    s.spec = fields;
    if (!check_spec(fields)) {
      discard_schema();
      return nullptr;
    }
  }
  g->ready = true;
  Py_RETURN_NONE;
}

// schema_marshal(obj, type name) -> marshalled dict tree
extern "C" PyObject* m2k_schema_marshal(PyObject* obj, PyObject* type_name) {
  if (g == nullptr || !g->ready) {
    PyErr_SetString(PyExc_RuntimeError, "schema_init was not called");
    return nullptr;
  }
  const char* tn = PyUnicode_AsUTF8(type_name);
  if (!tn) return nullptr;
  auto it = g->struct_index.find(tn);
  if (it == g->struct_index.end()) {
    PyErr_Format(PyExc_KeyError, "%s", tn);
    return nullptr;
  }
  return marshal_struct(obj, it->second);
}
