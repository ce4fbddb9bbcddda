/* Line-coverage tracer for scripts/coverage.py: a C trace function
 * (PyEval_SetTrace) that records, per source file under one directory
 * prefix, which lines ran.  No coverage package is installed here, and a
 * sys.settrace tracer in Python slows the suite several times over; this
 * one costs one pointer-keyed table probe per Python call and one bit set
 * per traced line.
 *
 * On every call event the frame's code object is looked up in an open
 * addressing table (the code objects are kept alive, so an address is
 * never reused while it is in the table).  Frames of code outside the
 * prefix get f_trace_lines = 0, so the interpreter sends no line events
 * for them at all; frames inside it set their line's bit in the file's
 * bitmap.  CPython 3.10 frame layout (cpython/frameobject.h).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <frameobject.h>
#include <string.h>

typedef struct {
    PyObject *code;   /* strong reference; NULL = empty slot */
    int file;         /* index into files[], -1 = outside the prefix */
} Slot;

typedef struct {
    PyObject *name;   /* str */
    unsigned char *bits;
    Py_ssize_t nbits;
} File;

static Slot *slots;
static Py_ssize_t nslots, nused;
static File *files;
static Py_ssize_t nfiles, capfiles;
static char *prefix;
static Py_ssize_t prefix_len;

static Py_ssize_t hash_ptr(PyObject *p) {
    size_t x = (size_t)p;
    x ^= x >> 17;
    x *= (size_t)0x9E3779B97F4A7C15ULL;
    return (Py_ssize_t)(x >> 7);
}

static int grow_table(void) {
    Py_ssize_t n = nslots ? nslots * 2 : 4096;
    Slot *t = PyMem_Calloc((size_t)n, sizeof(Slot));
    if (!t) return -1;
    for (Py_ssize_t i = 0; i < nslots; i++) {
        if (!slots[i].code) continue;
        Py_ssize_t j = hash_ptr(slots[i].code) & (n - 1);
        while (t[j].code) j = (j + 1) & (n - 1);
        t[j] = slots[i];
    }
    PyMem_Free(slots);
    slots = t;
    nslots = n;
    return 0;
}

static int file_index(PyObject *filename) {
    for (Py_ssize_t i = 0; i < nfiles; i++)
        if (PyUnicode_Compare(files[i].name, filename) == 0) return (int)i;
    if (nfiles == capfiles) {
        Py_ssize_t n = capfiles ? capfiles * 2 : 256;
        File *f = PyMem_Realloc(files, (size_t)n * sizeof(File));
        if (!f) return -1;
        files = f;
        capfiles = n;
    }
    Py_INCREF(filename);
    files[nfiles].name = filename;
    files[nfiles].bits = NULL;
    files[nfiles].nbits = 0;
    return (int)nfiles++;
}

/* -2 on error */
static int code_file(PyCodeObject *co) {
    if (nused * 2 >= nslots && grow_table() < 0) return -2;
    Py_ssize_t j = hash_ptr((PyObject *)co) & (nslots - 1);
    while (slots[j].code) {
        if (slots[j].code == (PyObject *)co) return slots[j].file;
        j = (j + 1) & (nslots - 1);
    }
    int idx = -1;
    Py_ssize_t len;
    const char *fn = PyUnicode_AsUTF8AndSize(co->co_filename, &len);
    if (!fn) { PyErr_Clear(); }
    else if (len >= prefix_len && memcmp(fn, prefix, (size_t)prefix_len) == 0) {
        idx = file_index(co->co_filename);
        if (idx < 0) return -2;
    }
    Py_INCREF(co);
    slots[j].code = (PyObject *)co;
    slots[j].file = idx;
    nused++;
    return idx;
}

static int mark(int idx, int line) {
    if (line <= 0) return 0;
    File *f = &files[idx];
    if (line >= f->nbits) {
        Py_ssize_t n = f->nbits ? f->nbits : 512;
        while (n <= line) n *= 2;
        unsigned char *b = PyMem_Realloc(f->bits, (size_t)n / 8);
        if (!b) return -1;
        memset(b + f->nbits / 8, 0, (size_t)(n - f->nbits) / 8);
        f->bits = b;
        f->nbits = n;
    }
    f->bits[line >> 3] |= (unsigned char)(1u << (line & 7));
    return 0;
}

static int tracer(PyObject *obj, PyFrameObject *frame, int what, PyObject *arg) {
    (void)obj; (void)arg;
    if (what == PyTrace_CALL) {
        int idx = code_file(frame->f_code);
        if (idx == -2) { PyErr_Clear(); return 0; }
        if (idx < 0) {
            frame->f_trace_lines = 0;
            return 0;
        }
        frame->f_trace_lines = 1;
        return 0;
    }
    if (what == PyTrace_LINE) {
        int idx = code_file(frame->f_code);
        if (idx >= 0 && mark(idx, PyFrame_GetLineNumber(frame)) < 0) PyErr_Clear();
    }
    return 0;
}

static PyObject *py_start(PyObject *self, PyObject *args) {
    (void)self; (void)args;
    if (!prefix) {
        PyErr_SetString(PyExc_RuntimeError, "linecov: set_prefix first");
        return NULL;
    }
    PyEval_SetTrace(tracer, NULL);
    Py_RETURN_NONE;
}

static PyObject *py_stop(PyObject *self, PyObject *args) {
    (void)self; (void)args;
    PyEval_SetTrace(NULL, NULL);
    Py_RETURN_NONE;
}

static PyObject *py_set_prefix(PyObject *self, PyObject *args) {
    (void)self;
    const char *p;
    Py_ssize_t n;
    if (!PyArg_ParseTuple(args, "s#", &p, &n)) return NULL;
    char *c = PyMem_Malloc((size_t)n + 1);
    if (!c) return PyErr_NoMemory();
    memcpy(c, p, (size_t)n);
    c[n] = 0;
    PyMem_Free(prefix);
    prefix = c;
    prefix_len = n;
    Py_RETURN_NONE;
}

/* {filename: [line, ...]} of every line that ran */
static PyObject *py_data(PyObject *self, PyObject *args) {
    (void)self; (void)args;
    PyObject *out = PyDict_New();
    if (!out) return NULL;
    for (Py_ssize_t i = 0; i < nfiles; i++) {
        PyObject *lines = PyList_New(0);
        if (!lines) { Py_DECREF(out); return NULL; }
        for (Py_ssize_t l = 0; l < files[i].nbits; l++) {
            if (files[i].bits[l >> 3] & (1u << (l & 7))) {
                PyObject *v = PyLong_FromSsize_t(l);
                if (!v || PyList_Append(lines, v) < 0) { Py_XDECREF(v); Py_DECREF(lines); Py_DECREF(out); return NULL; }
                Py_DECREF(v);
            }
        }
        if (PyDict_SetItem(out, files[i].name, lines) < 0) { Py_DECREF(lines); Py_DECREF(out); return NULL; }
        Py_DECREF(lines);
    }
    return out;
}

static PyMethodDef methods[] = {
    {"set_prefix", py_set_prefix, METH_VARARGS, "Trace only code whose file name starts with this."},
    {"start", py_start, METH_NOARGS, "Start tracing the calling thread."},
    {"stop", py_stop, METH_NOARGS, "Stop tracing the calling thread."},
    {"data", py_data, METH_NOARGS, "{filename: [lines that ran]}."},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "m2k_linecov", NULL, -1, methods};

PyMODINIT_FUNC PyInit_m2k_linecov(void) { return PyModule_Create(&moddef); }
