/* Low-overhead Python -> C-ABI call path for libmvae_hip.so (host side of the boundary, x86-64 SysV only).
 *
 * ctypes spends ~3-5 us per call converting arguments through `argtypes`; the small-batch training steps make
 * ~400 such calls per step (c3: ~1.5 ms of host time). This module registers each entry point once -- its address
 * (from the ctypes handle) and its signature string, the same type codes as _lib.SIGNATURES -- and calls it through
 * one fixed trampoline: integer-class arguments (pointers, int, long long, size_t, uint64) go to the six integer
 * registers and then to the stack in declaration order, float-class arguments (float, double) to xmm0-7, exactly as
 * the SysV calling convention places them. Extra trailing register / stack arguments are ignored by the callee (the
 * caller owns the stack), so one prototype with 6 + 8 + 26 slots serves every signature with at most 8 float-class
 * and 32 integer-class arguments; registration refuses anything else (that entry point stays on ctypes).
 *
 *   bind(addr, sig) -> index      sig: return code then argument codes, e.g. "IPPPIF" (I int, L long long,
 *                                 Z size_t, U uint64, P pointer, F float, D double; return I or Z)
 *   call(index, *args) -> int     raises TypeError on a bad argument; the status code is checked by the caller
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

#define MAX_FN 256
#define MAX_ARGS 40
#define N_STACK 26

typedef int64_t (*tramp_t)(int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, double, double, double, double,
                           double, double, double, double, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                           int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                           int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t);

typedef struct {
  void* fn;
  char ret;
  int nargs;
  char code[MAX_ARGS];
} entry_t;

static entry_t g_fn[MAX_FN];
static int g_nfn = 0;

static PyObject* fast_bind(PyObject* self, PyObject* args) {
  unsigned long long addr;
  const char* sig;
  if (!PyArg_ParseTuple(args, "Ks", &addr, &sig)) return NULL;
#if !(defined(__x86_64__) && defined(__linux__))
  Py_RETURN_NONE; /* the trampoline assumes the x86-64 SysV argument placement: other hosts stay on ctypes */
#endif
  const int n = (int)strlen(sig) - 1;
  if (n < 0 || n > MAX_ARGS || g_nfn >= MAX_FN || (sig[0] != 'I' && sig[0] != 'Z')) Py_RETURN_NONE;
  int ni = 0, nf = 0;
  for (int i = 0; i < n; ++i) {
    const char c = sig[1 + i];
    if (c == 'F' || c == 'D') ++nf;
    else if (c == 'I' || c == 'L' || c == 'Z' || c == 'U' || c == 'P') ++ni;
    else Py_RETURN_NONE;
  }
  if (nf > 8 || ni > 6 + N_STACK) Py_RETURN_NONE;
  entry_t* e = &g_fn[g_nfn];
  e->fn = (void*)(uintptr_t)addr;
  e->ret = sig[0];
  e->nargs = n;
  memcpy(e->code, sig + 1, (size_t)n);
  return PyLong_FromLong(g_nfn++);
}

static PyObject* fast_call(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs < 1) {
    PyErr_SetString(PyExc_TypeError, "call(index, *args)");
    return NULL;
  }
  const long idx = PyLong_AsLong(args[0]);
  if (idx < 0 || idx >= g_nfn) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_IndexError, "unbound entry point");
    return NULL;
  }
  const entry_t* e = &g_fn[idx];
  if (nargs - 1 != e->nargs) {
    PyErr_Format(PyExc_TypeError, "expected %d arguments, got %zd", e->nargs, nargs - 1);
    return NULL;
  }
  int64_t iv[6 + N_STACK];
  double fv[8];
  memset(iv, 0, sizeof(iv));
  memset(fv, 0, sizeof(fv));
  int ni = 0, nf = 0;
  for (int i = 0; i < e->nargs; ++i) {
    PyObject* o = args[1 + i];
    const char c = e->code[i];
    if (c == 'F' || c == 'D') {
      const double d = PyFloat_AsDouble(o);
      if (d == -1.0 && PyErr_Occurred()) return NULL;
      if (c == 'F') {  // a float argument lives in the low 32 bits of its xmm register
        union { float f; uint32_t u; } fb;
        union { uint64_t u; double d; } db;
        fb.f = (float)d;
        db.u = (uint64_t)fb.u;
        fv[nf++] = db.d;
      } else {
        fv[nf++] = d;
      }
    } else if (c == 'P') {
      if (o == Py_None) {
        iv[ni++] = 0;
      } else {
        const unsigned long long p = PyLong_AsUnsignedLongLongMask(o);
        if (PyErr_Occurred()) return NULL;
        iv[ni++] = (int64_t)p;
      }
    } else if (c == 'U' || c == 'Z') {
      const unsigned long long u = PyLong_AsUnsignedLongLongMask(o);
      if (PyErr_Occurred()) return NULL;
      iv[ni++] = (int64_t)u;
    } else {  /* I, L */
      const long long v = PyLong_AsLongLong(o);
      if (v == -1 && PyErr_Occurred()) return NULL;
      iv[ni++] = (c == 'I') ? (int64_t)(int32_t)v : (int64_t)v;
    }
  }
  const tramp_t f = (tramp_t)e->fn;
  int64_t r;
  Py_BEGIN_ALLOW_THREADS
  r = f(iv[0], iv[1], iv[2], iv[3], iv[4], iv[5], fv[0], fv[1], fv[2], fv[3], fv[4], fv[5], fv[6], fv[7], iv[6],
        iv[7], iv[8], iv[9], iv[10], iv[11], iv[12], iv[13], iv[14], iv[15], iv[16], iv[17], iv[18], iv[19], iv[20],
        iv[21], iv[22], iv[23], iv[24], iv[25], iv[26], iv[27], iv[28], iv[29], iv[30], iv[31]);
  Py_END_ALLOW_THREADS
  if (e->ret == 'I') return PyLong_FromLong((long)(int32_t)r);
  return PyLong_FromUnsignedLongLong((unsigned long long)r);
}

static PyMethodDef methods[] = {
    {"bind", (PyCFunction)fast_bind, METH_VARARGS, "bind(addr, sig) -> index or None"},
    {"call", (PyCFunction)(void (*)(void))fast_call, METH_FASTCALL, "call(index, *args) -> return value"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mvae_fast", NULL, -1, methods};

PyMODINIT_FUNC PyInit__mvae_fast(void) { return PyModule_Create(&module); }
