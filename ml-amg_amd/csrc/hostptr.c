/* Host-side helper of the batched amg_2_v entry (mlamg.multigrid.amg_2_v_batch): the data
 * pointers of many host buffers (numpy arrays) in one call. Filling mlamg_amg2v_problem
 * records needs eight pointers per problem; numpy's per-array accessors (.ctypes.data,
 * __array_interface__) cost 1.5-2.5 us each, which at 256 problems is milliseconds of a
 * ~10 ms farm. Plain CPython buffer protocol, no numpy headers; no device code. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

/* data_ptrs(seq, out): out[i] = address of seq[i]'s C-contiguous buffer (out: a writable
 * buffer of >= len(seq) uint64). The buffers must stay alive while the addresses are used. */
static PyObject* data_ptrs(PyObject* self, PyObject* args) {
  (void)self;
  PyObject* seq;
  Py_buffer out;
  if (!PyArg_ParseTuple(args, "Ow*", &seq, &out)) return NULL;
  PyObject* fast = PySequence_Fast(seq, "data_ptrs: a sequence of buffers is required");
  if (!fast) {
    PyBuffer_Release(&out);
    return NULL;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  if (out.len < (Py_ssize_t)sizeof(uint64_t) * n) {
    Py_DECREF(fast);
    PyBuffer_Release(&out);
    PyErr_SetString(PyExc_ValueError, "data_ptrs: output buffer too small");
    return NULL;
  }
  uint64_t* o = (uint64_t*)out.buf;
  PyObject** items = PySequence_Fast_ITEMS(fast);
  for (Py_ssize_t i = 0; i < n; ++i) {
    Py_buffer v;
    if (PyObject_GetBuffer(items[i], &v, PyBUF_C_CONTIGUOUS) != 0) {
      Py_DECREF(fast);
      PyBuffer_Release(&out);
      return NULL;
    }
    o[i] = (uint64_t)(uintptr_t)v.buf;
    PyBuffer_Release(&v);
  }
  Py_DECREF(fast);
  PyBuffer_Release(&out);
  Py_RETURN_NONE;
}

static PyMethodDef methods[] = {
    {"data_ptrs", data_ptrs, METH_VARARGS, "data_ptrs(seq, out): buffer addresses into out"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_hostptr", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__hostptr(void) { return PyModule_Create(&module); }
