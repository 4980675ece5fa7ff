/* Host-memory boundary of the list API: Python objects <-> flat buffers, in one C pass.
 *
 * The reference's crypters take and return Python lists (`_secagg_crypter.py:45-230`):
 * List[float] model parameters into encrypt, List[int] 2048-bit JL ciphertexts out of it
 * and, per party, back into aggregate.  Converting those lists element by element in Python
 * (array('d', ...), int.to_bytes / int.from_bytes per ciphertext) cost about as much host
 * time as the GPU spends on a model-sized encrypt (end-to-end).  These
 * three loops do the same conversions without an intermediate Python object per element:
 *
 *   floats_to_f64(list, out)        -> -1, or the index of the first non-float item
 *                                      (isinstance(v, float) semantics: subclasses pass)
 *   ints_to_bytes(list, n, out)     -> -1, or the index of the first item that is not an
 *                                      int in [0, 2^(8n)) (the caller then takes its slow
 *                                      path: type error or reduction mod N^2)
 *   bytes_to_ints(buf, n)           -> list of the unsigned little-endian n-byte integers
 *
 * `out` is any writable C-contiguous buffer (a numpy array) of the exact size.  Host code,
 * not part of the GPU compute path: the arithmetic stays in the HIP library.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <longintrepr.h>
#include <stdint.h>
#include <string.h>

/* Non-negative int -> nb little-endian bytes (nb a multiple of 4) straight from CPython's
 * 30-bit digits; 0 on success, -1 if negative or too wide.  _PyLong_AsByteArray gives the
 * same bytes but goes byte by byte (~4x slower on 2048-bit values). */
static int long_to_words(PyLongObject* v, unsigned char* dst, Py_ssize_t nb) {
    Py_ssize_t size = Py_SIZE(v);
    if (size < 0) return -1;
    uint32_t* w = (uint32_t*)dst; /* caller's buffer: 4-byte aligned numpy rows */
    Py_ssize_t nw = nb / 4, k = 0;
    uint64_t acc = 0;
    int bits = 0;
    for (Py_ssize_t i = 0; i < size; ++i) {
        acc |= (uint64_t)v->ob_digit[i] << bits;
        bits += PyLong_SHIFT;
        while (bits >= 32) {
            if (k == nw) return -1;
            w[k++] = (uint32_t)acc;
            acc >>= 32;
            bits -= 32;
        }
    }
    if (bits > 0 && acc) {
        if (k == nw) return -1;
        w[k++] = (uint32_t)acc;
    }
    if (k == nw && acc >> 32) return -1;
    memset(w + k, 0, (size_t)(nw - k) * 4);
    return 0;
}

static int get_out(PyObject* obj, Py_buffer* view, Py_ssize_t need) {
    if (PyObject_GetBuffer(obj, view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0) return -1;
    if (view->len != need) {
        PyErr_Format(PyExc_ValueError, "output buffer holds %zd bytes, %zd needed", view->len, need);
        PyBuffer_Release(view);
        return -1;
    }
    return 0;
}

static PyObject* floats_to_f64(PyObject* self, PyObject* args) {
    PyObject *seq, *out;
    if (!PyArg_ParseTuple(args, "O!O", &PyList_Type, &seq, &out)) return NULL;
    Py_ssize_t n = PyList_GET_SIZE(seq);
    Py_buffer view;
    if (get_out(out, &view, n * (Py_ssize_t)sizeof(double)) < 0) return NULL;
    double* dst = (double*)view.buf;
    Py_ssize_t bad = -1;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* v = PyList_GET_ITEM(seq, i);
        if (!PyFloat_Check(v)) {
            bad = i;
            break;
        }
        dst[i] = PyFloat_AS_DOUBLE(v);
    }
    PyBuffer_Release(&view);
    return PyLong_FromSsize_t(bad);
}

static PyObject* ints_to_bytes(PyObject* self, PyObject* args) {
    PyObject *seq, *out;
    Py_ssize_t nb;
    if (!PyArg_ParseTuple(args, "O!nO", &PyList_Type, &seq, &nb, &out)) return NULL;
    if (nb <= 0) {
        PyErr_SetString(PyExc_ValueError, "width must be positive");
        return NULL;
    }
    Py_ssize_t n = PyList_GET_SIZE(seq);
    Py_buffer view;
    if (get_out(out, &view, n * nb) < 0) return NULL;
    unsigned char* dst = (unsigned char*)view.buf;
    int words = nb % 4 == 0 && ((uintptr_t)dst & 3) == 0;
    Py_ssize_t bad = -1;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* v = PyList_GET_ITEM(seq, i);
        int rc = !PyLong_Check(v) ? -1
                 : words ? long_to_words((PyLongObject*)v, dst + i * nb, nb)
                         : _PyLong_AsByteArray((PyLongObject*)v, dst + i * nb, (size_t)nb, 1, 0);
        if (rc < 0) {
            PyErr_Clear(); /* OverflowError (negative or too wide): the caller's slow path */
            bad = i;
            break;
        }
    }
    PyBuffer_Release(&view);
    return PyLong_FromSsize_t(bad);
}

static PyObject* bytes_to_ints(PyObject* self, PyObject* args) {
    Py_buffer view;
    Py_ssize_t nb;
    if (!PyArg_ParseTuple(args, "y*n", &view, &nb)) return NULL;
    if (nb <= 0 || view.len % nb) {
        PyBuffer_Release(&view);
        PyErr_SetString(PyExc_ValueError, "buffer is not a whole number of values");
        return NULL;
    }
    Py_ssize_t n = view.len / nb;
    PyObject* lst = PyList_New(n);
    if (lst) {
        const unsigned char* src = (const unsigned char*)view.buf;
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject* v = _PyLong_FromByteArray(src + i * nb, (size_t)nb, 1, 0);
            if (!v) {
                Py_CLEAR(lst);
                break;
            }
            PyList_SET_ITEM(lst, i, v);
        }
    }
    PyBuffer_Release(&view);
    return lst;
}

static PyMethodDef methods[] = {
    {"floats_to_f64", floats_to_f64, METH_VARARGS, "list of floats -> float64 buffer; -1 or first bad index"},
    {"ints_to_bytes", ints_to_bytes, METH_VARARGS, "list of ints -> n-byte LE unsigned; -1 or first bad index"},
    {"bytes_to_ints", bytes_to_ints, METH_VARARGS, "buffer of n-byte LE unsigned values -> list of ints"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fbm_pyconv", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fbm_pyconv(void) { return PyModule_Create(&module); }
