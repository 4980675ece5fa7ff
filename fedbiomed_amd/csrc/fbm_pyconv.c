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
 *   ints_to_bytes_held(lists, lo, hi, n, out)
 *                                   -> items [lo, hi) of every list into out [len(lists), hi - lo, n]
 *                                      on host threads in one call that holds the GIL: the readers need
 *                                      no pins (see there); -1 or the first bad flat index (list u,
 *                                      item i: u (hi - lo) + i)
 *   none_list(n)                    -> [None] * n (the output list that f64_into_list fills)
 *   float_pool(n)                   -> n fresh 0.0 floats: an output list made ahead, filled in place
 *   f64_into_list(list, offset, buf) -> list[offset:offset + len(buf)] = floats of the float64 buffer
 *   set_conv_threads(t)             -> the threaded loops' default host-thread count (returns the old one)
 *   all_ints_lists(lists)           -> -1, or the first list holding a non-int (every list in one pass)
 *   int_pool(n, nb)                 -> n fresh ints with room for nb-byte values: an output list made ahead
 *   words_into_pool(pool, buf, nb[, off]) -> the pool's ints [off, ...) take buf's values in place
 *
 * `out` is any writable C-contiguous buffer (a numpy array) of the exact size.  Host code,
 * not part of the GPU compute path: the arithmetic stays in the HIP library.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#if PY_VERSION_HEX < 0x030B0000
#include <longintrepr.h> /* 3.11 moved it to cpython/longintrepr.h, which Python.h includes */
#endif
#include <pthread.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

/* The digit-level fast paths read CPython's PyLongObject layout (ob_digit, Py_SIZE as the
 * signed digit count), which is the layout of 3.10 and 3.11 (the versions this module is built and
 * tested on); 3.12 changed it (long_value.ob_digit, lv_tag).  On any other version the conversions
 * go through the byte-array API instead, on one thread. */
#ifndef FBM_DIGITS_FAST /* -DFBM_DIGITS_FAST=0 builds the portable path on any version (tested) */
#if PY_VERSION_HEX >= 0x030A0000 && PY_VERSION_HEX < 0x030C0000
#define FBM_DIGITS_FAST 1
#else
#define FBM_DIGITS_FAST 0
#endif
#endif

/* In-place writes into objects the module made and nothing else holds yet -- a float_pool float's
 * ob_fval, an int_pool int's digits -- only on 3.10 / 3.11 (or -DFBM_INPLACE=0: never, tested).  Off, a
 * pool float is replaced by a new float (its release frees it before the list is returned) and there
 * are no int pools: every output object is made with its value. */
#ifndef FBM_INPLACE
#define FBM_INPLACE FBM_DIGITS_FAST
#endif

#if FBM_DIGITS_FAST
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
#endif

/* Non-negative int -> nb little-endian bytes through the public/stable byte API (any
 * version; the GIL must be held: it may set an exception, which is cleared). */
static int long_to_bytes_api(PyObject* v, unsigned char* dst, Py_ssize_t nb) {
    if (_PyLong_Sign(v) < 0) return -1;
#if PY_VERSION_HEX >= 0x030D0000
    Py_ssize_t need = PyLong_AsNativeBytes(v, dst, nb, Py_ASNATIVEBYTES_LITTLE_ENDIAN | Py_ASNATIVEBYTES_UNSIGNED_BUFFER);
    if (need < 0) {
        PyErr_Clear();
        return -1;
    }
    return need <= nb ? 0 : -1;
#else
    int rc = _PyLong_AsByteArray((PyLongObject*)v, dst, (size_t)nb, 1, 0);
    if (rc < 0) PyErr_Clear();
    return rc;
#endif
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

/* floats -> float64 over [lo, hi) of the list's item array: stops at its first non-float */
typedef struct {
    PyObject** items;
    double* dst;
    Py_ssize_t lo, hi, bad;
} fconv_job;

static void* fconv_range(void* arg) {
    fconv_job* j = (fconv_job*)arg;
    j->bad = -1;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
        PyObject* v = j->items[i];
        if (!PyFloat_Check(v)) {
            j->bad = i;
            break;
        }
        j->dst[i] = PyFloat_AS_DOUBLE(v);
    }
    return NULL;
}

/* Host threads of the threaded loops: FBM_CONV_THREADS when set, else the default the Python side
 * sets once from the process's CPU share (its affinity, capped by a cgroup quota; at most 16,
 * fedbiomed_amd/_device.py:host_cpu_share), else 8. */
static long g_default_threads = 8;

static PyObject* set_conv_threads(PyObject* self, PyObject* args) {
    long t;
    if (!PyArg_ParseTuple(args, "l", &t)) return NULL;
    long old = g_default_threads;
    g_default_threads = t < 1 ? 1 : t > 64 ? 64 : t;
    return PyLong_FromLong(old);
}

static int conv_threads(Py_ssize_t n) {
    const char* e = getenv("FBM_CONV_THREADS");
    long t = e ? strtol(e, NULL, 10) : g_default_threads;
    if (t < 1) t = 1;
    if (t > 64) t = 64;
    if (t > n / 1024) t = n / 1024 > 0 ? (long)(n / 1024) : 1;
    return (int)t;
}

/* Large lists are read by several threads WHILE THIS THREAD HOLDS THE GIL: no Python code runs
 * meanwhile, so the list and its items cannot change or be freed under the readers (they touch
 * no interpreter state: the float objects' type pointers and values, and the type objects'
 * MRO for a float subclass), and no reference needs to be taken per item.  ~10 M floats of a
 * model update: one thread ~15 ms, dominated by the scattered object reads. */
#define FCONV_PAR_MIN (1 << 20)

static PyObject* floats_to_f64(PyObject* self, PyObject* args) {
    PyObject *seq, *out;
    if (!PyArg_ParseTuple(args, "O!O", &PyList_Type, &seq, &out)) return NULL;
    Py_ssize_t n = PyList_GET_SIZE(seq);
    Py_buffer view;
    if (get_out(out, &view, n * (Py_ssize_t)sizeof(double)) < 0) return NULL;
    double* dst = (double*)view.buf;
    PyObject** items = ((PyListObject*)seq)->ob_item;
    int nt = n >= FCONV_PAR_MIN ? conv_threads(n) : 1;
    fconv_job jobs[64];
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (fconv_job){items, dst, n * t / nt, n * (t + 1) / nt, -1};
        if (t > 0) started[t] = pthread_create(&tid[t], NULL, fconv_range, &jobs[t]) == 0;
    }
    fconv_range(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            fconv_range(&jobs[t]); /* thread creation failed: its range here */
    }
    Py_ssize_t bad = -1;
    for (int t = 0; t < nt && bad < 0; ++t) bad = jobs[t].bad;
    PyBuffer_Release(&view);
    return PyLong_FromSsize_t(bad);
}

/* Ciphertext-sized conversions run on several host threads WHILE THIS THREAD HOLDS THE GIL (as
 * floats_to_f64): no Python code runs meanwhile, so the list cannot change and its ints cannot be
 * freed under the readers, which read only the ints' digits (immutable; long_to_words touches no
 * interpreter state) -- no reference per item is needed.  (Round 4's form released the GIL and pinned
 * every item first: a reference taken and dropped on this thread, ~10 ns each, a third of the
 * conversion's own cost.)  Thread count: conv_threads above. */
#define PAR_MIN_BYTES (1 << 20)

typedef struct {
    PyObject** items;
    unsigned char* dst;
    Py_ssize_t lo, hi, nb, bad;
} conv_job;

#if FBM_DIGITS_FAST
static void* conv_range(void* arg) {
    conv_job* j = (conv_job*)arg;
    j->bad = -1;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
        PyObject* v = j->items[i];
        if (!PyLong_Check(v) || long_to_words((PyLongObject*)v, j->dst + i * j->nb, j->nb) < 0) {
            j->bad = i;
            break;
        }
    }
    return NULL;
}


/* -1, or the first bad index over all ranges (each range stops at its own first bad item). */
static Py_ssize_t ints_to_words_parallel(PyObject* seq, Py_ssize_t n, Py_ssize_t nb, unsigned char* dst,
                                         int nt) {
    PyObject** items = ((PyListObject*)seq)->ob_item;
    conv_job jobs[64];
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (conv_job){items, dst, n * t / nt, n * (t + 1) / nt, nb, -1};
        if (t > 0) started[t] = pthread_create(&tid[t], NULL, conv_range, &jobs[t]) == 0;
    }
    conv_range(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            conv_range(&jobs[t]); /* thread creation failed: do its range here */
    }
    Py_ssize_t bad = -1;
    for (int t = 0; t < nt && bad < 0; ++t) bad = jobs[t].bad;
    return bad;
}
#endif

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
    Py_ssize_t bad = -1;
#if FBM_DIGITS_FAST
    int words = nb % 4 == 0 && ((uintptr_t)dst & 3) == 0;
    int nt = words && n * nb >= PAR_MIN_BYTES ? conv_threads(n) : 1;
#else
    int words = 0, nt = 1;
#endif
    if (nt > 1) {
#if FBM_DIGITS_FAST
        bad = ints_to_words_parallel(seq, n, nb, dst, nt);
#endif
    } else {
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject* v = PyList_GET_ITEM(seq, i);
            int rc = -1;
            if (PyLong_Check(v)) {
#if FBM_DIGITS_FAST
                rc = words ? long_to_words((PyLongObject*)v, dst + i * nb, nb) : long_to_bytes_api(v, dst + i * nb, nb);
#else
                (void)words;
                rc = long_to_bytes_api(v, dst + i * nb, nb);
#endif
            }
            if (rc < 0) { /* negative, too wide or not an int: the caller's slow path */
                bad = i;
                break;
            }
        }
    }
    PyBuffer_Release(&view);
    return PyLong_FromSsize_t(bad);
}

static PyObject* long_from_bytes_api(const unsigned char* src, Py_ssize_t nb) {
#if PY_VERSION_HEX >= 0x030D0000
    return PyLong_FromUnsignedNativeBytes(src, (size_t)nb, Py_ASNATIVEBYTES_LITTLE_ENDIAN);
#else
    return _PyLong_FromByteArray(src, (size_t)nb, 1, 0);
#endif
}

#if FBM_DIGITS_FAST
/* nw little-endian 32-bit words -> int, built straight in CPython's 30-bit digits
 * (_PyLong_FromByteArray goes byte by byte).  Split in two so that a long list is made in two
 * passes: this thread allocates every object (the allocator is the interpreter's), then host
 * threads write the digits of the objects nobody else has seen yet (pure arithmetic). */
static Py_ssize_t words_used(const uint32_t* w, Py_ssize_t nw) {
    while (nw > 0 && w[nw - 1] == 0) --nw;
    return nw;
}

/* An int of nw significant words: the small ones (nw <= 1, the small-int cache among them) made
 * whole, the others allocated with their digits left for long_fill. */
static PyObject* long_alloc(const uint32_t* w, Py_ssize_t nw) {
    if (nw <= 1) return PyLong_FromUnsignedLong(nw ? w[0] : 0);
    Py_ssize_t nbits = 32 * (nw - 1) + (32 - __builtin_clz(w[nw - 1]));
    return (PyObject*)_PyLong_New((nbits + PyLong_SHIFT - 1) / PyLong_SHIFT);
}

static void long_fill(PyLongObject* v, const uint32_t* w, Py_ssize_t nw) {
    const Py_ssize_t nd = Py_SIZE(v);
    uint64_t acc = 0;
    int bits = 0;
    Py_ssize_t k = 0, d = 0;
    while (d < nd) {
        if (bits < PyLong_SHIFT && k < nw) {
            acc |= (uint64_t)w[k++] << bits;
            bits += 32;
        }
        v->ob_digit[d++] = (digit)(acc & PyLong_MASK);
        acc >>= PyLong_SHIFT;
        bits -= PyLong_SHIFT;
    }
}

typedef struct {
    PyObject** items;
    const unsigned char* src;
    Py_ssize_t lo, hi, nb;
} fill_job;

static void* fill_range(void* arg) {
    fill_job* j = (fill_job*)arg;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
        const uint32_t* w = (const uint32_t*)(j->src + i * j->nb);
        Py_ssize_t nw = words_used(w, j->nb / 4);
        if (nw > 1) long_fill((PyLongObject*)j->items[i], w, nw);
    }
    return NULL;
}

/* n values of nb bytes (nb % 4 == 0, src 4-byte aligned) into the NULL-initialised list: 0, or -1 with
 * an exception set (the items made so far stay in the list, their digits unread by anyone). */
static int words_into_list(PyObject* lst, const unsigned char* src, Py_ssize_t n, Py_ssize_t nb) {
    PyObject** items = ((PyListObject*)lst)->ob_item;
    for (Py_ssize_t i = 0; i < n; ++i) {
        const uint32_t* w = (const uint32_t*)(src + i * nb);
        if (!(items[i] = long_alloc(w, words_used(w, nb / 4)))) return -1;
    }
    int nt = n * nb >= PAR_MIN_BYTES ? conv_threads(n) : 1;
    fill_job jobs[64];
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (fill_job){items, src, n * t / nt, n * (t + 1) / nt, nb};
        if (t > 0) started[t] = pthread_create(&tid[t], NULL, fill_range, &jobs[t]) == 0;
    }
    fill_range(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            fill_range(&jobs[t]);
    }
    return 0;
}
#endif

/* The list is made by this thread; for the word layout the digits are written by host threads
 * once every object exists, while this thread holds the GIL and before the list is returned: no
 * other code can see an object whose digits are still being written. */
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
#if FBM_DIGITS_FAST
        if (nb % 4 == 0 && ((uintptr_t)src & 3) == 0) {
            if (words_into_list(lst, src, n, nb) < 0) Py_CLEAR(lst);
            PyBuffer_Release(&view);
            return lst;
        }
#endif
        for (Py_ssize_t i = 0; i < n; ++i) {
            PyObject* v = long_from_bytes_api(src + i * nb, nb);
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

/* all(isinstance(v, int) for v in seq) for a list: PyLong_Check per item (int subclasses, bool among
 * them, count as the reference's isinstance does) -- no per-item hashing, unlike set(map(type, seq)). */
typedef struct {
    PyObject** items;
    Py_ssize_t lo, hi;
    int ok;
} intchk_job;

static void* intchk_range(void* arg) {
    intchk_job* j = (intchk_job*)arg;
    j->ok = 1;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i)
        if (!PyLong_Check(j->items[i])) {
            j->ok = 0;
            break;
        }
    return NULL;
}

/* Large lists are checked by several threads while this one holds the GIL (as floats_to_f64: the
 * readers touch only the items' type pointers): a party's 333 334 ciphertexts are ~1.3 ms of
 * scattered reads on one thread. */
static PyObject* all_ints(PyObject* self, PyObject* args) {
    PyObject* seq;
    if (!PyArg_ParseTuple(args, "O!", &PyList_Type, &seq)) return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(seq);
    PyObject** items = ((PyListObject*)seq)->ob_item;
    int nt = n >= (1 << 16) ? conv_threads(n) : 1;
    if (nt > 4) nt = 4;
    intchk_job jobs[4];
    pthread_t tid[4];
    int started[4] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (intchk_job){items, n * t / nt, n * (t + 1) / nt, 1};
        if (t > 0) started[t] = pthread_create(&tid[t], NULL, intchk_range, &jobs[t]) == 0;
    }
    intchk_range(&jobs[0]);
    int ok = jobs[0].ok;
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            intchk_range(&jobs[t]);
        ok &= jobs[t].ok;
    }
    return PyBool_FromLong(ok);
}

/* The output list's slots: None (a none_list) or exact floats (a float_pool).  Writing value d into a
 * slot: None -> a new float; a float only this list holds (reference count 1, made by float_pool and
 * never handed out) -> its value overwritten in place, no allocation (the object is not yet visible to
 * any Python code: the list is returned only once filled); a float someone else also holds -> replaced
 * by a new one (its release cannot free it, so no destructor runs mid-loop).  Anything else refused. */
static int check_slots(PyObject* const* items, Py_ssize_t k) {
    for (Py_ssize_t i = 0; i < k; ++i)
        if (items[i] != Py_None && !PyFloat_CheckExact(items[i])) {
            PyErr_SetString(PyExc_ValueError, "f64_into_list fills slots that hold None or floats only");
            return -1;
        }
    return 0;
}

static int fill_slots(PyObject** items, const double* src, Py_ssize_t k) {
    for (Py_ssize_t i = 0; i < k; ++i) {
        PyObject* o = items[i];
        if (FBM_INPLACE && o != Py_None && Py_REFCNT(o) == 1) {
            ((PyFloatObject*)o)->ob_fval = src[i];
            continue;
        }
        PyObject* v = PyFloat_FromDouble(src[i]);
        if (!v) return -1;
        items[i] = v;
        Py_DECREF(o); /* None, a float with another holder, or (FBM_INPLACE off) a pool float: a float's
                         deallocation runs no Python code */
    }
    return 0;
}

static PyObject* make_none_list(Py_ssize_t n) {
    PyObject* lst = PyList_New(n);
    if (!lst) return NULL;
    PyObject** items = ((PyListObject*)lst)->ob_item;
    for (Py_ssize_t i = 0; i < n; ++i) {
        Py_INCREF(Py_None);
        items[i] = Py_None;
    }
    return lst;
}

/* The researcher aggregate's ciphertext conversion, one call per stripe: worker threads convert items
 * [lo, hi) of every party's list into `out` [P, hi - lo, nb] while this thread waits, the GIL held
 * throughout.  As the GIL is never released, no Python code runs until the call returns: no list can
 * change and no int be freed under the readers, so nothing is pinned (ints_to_bytes, which releases the
 * GIL, pays a reference per item, taken and dropped on this thread: ~10 ns each, a third of the
 * conversion's own cost).  The readers touch only the ints' digits and `out`.  Returns -1 or the first
 * bad flat index (u (hi - lo) + i). */
typedef struct {
    PyObject*** rows; /* each party's ob_item + lo */
    Py_ssize_t m, lo, hi, nb, bad;
    unsigned char* dst;
} heldconv_job;

#if FBM_DIGITS_FAST
static void* heldconv_range(void* arg) {
    heldconv_job* j = (heldconv_job*)arg;
    j->bad = -1;
    for (Py_ssize_t f = j->lo; f < j->hi; ++f) {
        PyObject* v = j->rows[f / j->m][f % j->m];
        if (!PyLong_Check(v) || long_to_words((PyLongObject*)v, j->dst + f * j->nb, j->nb) < 0) {
            j->bad = f;
            break;
        }
    }
    return NULL;
}
#endif

static PyObject* ints_to_bytes_held(PyObject* self, PyObject* args) {
    PyObject *lists, *out;
    Py_ssize_t lo, hi, nb;
    if (!PyArg_ParseTuple(args, "O!nnnO", &PyList_Type, &lists, &lo, &hi, &nb, &out)) return NULL;
    const Py_ssize_t P = PyList_GET_SIZE(lists), m = hi - lo;
    if (nb <= 0 || nb % 4 || lo < 0 || m < 0) {
        PyErr_SetString(PyExc_ValueError, "bad range or width (a positive multiple of 4 bytes)");
        return NULL;
    }
    for (Py_ssize_t u = 0; u < P; ++u) {
        PyObject* l = PyList_GET_ITEM(lists, u);
        if (!PyList_Check(l) || PyList_GET_SIZE(l) < hi) {
            PyErr_SetString(PyExc_ValueError, "every item must be a list holding the range");
            return NULL;
        }
    }
    Py_buffer oview;
    if (get_out(out, &oview, P * m * nb) < 0) return NULL;
    if (((uintptr_t)oview.buf & 3) != 0) {
        PyBuffer_Release(&oview);
        PyErr_SetString(PyExc_ValueError, "output buffer must be 4-byte aligned");
        return NULL;
    }
    PyObject*** rows = (PyObject***)PyMem_Malloc((size_t)(P > 0 ? P : 1) * sizeof(PyObject**));
    if (!rows) {
        PyBuffer_Release(&oview);
        return PyErr_NoMemory();
    }
    for (Py_ssize_t u = 0; u < P; ++u) rows[u] = ((PyListObject*)PyList_GET_ITEM(lists, u))->ob_item + lo;
    const Py_ssize_t n = P * m;
    Py_ssize_t bad = -1;
#if FBM_DIGITS_FAST
    int nt = n >= 1024 ? conv_threads(n) : 1;
    heldconv_job jobs[64];
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (heldconv_job){rows, m > 0 ? m : 1, n * t / nt, n * (t + 1) / nt, nb, -1, (unsigned char*)oview.buf};
        started[t] = t > 0 && pthread_create(&tid[t], NULL, heldconv_range, &jobs[t]) == 0;
    }
    heldconv_range(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            heldconv_range(&jobs[t]); /* thread creation failed: its range here */
    }
    for (int t = 0; t < nt && bad < 0; ++t) bad = jobs[t].bad;
#else /* the byte API: on this thread */
    for (Py_ssize_t f = 0; f < n && bad < 0; ++f) {
        PyObject* v = rows[f / m][f % m];
        if (!PyLong_Check(v) || long_to_bytes_api(v, (unsigned char*)oview.buf + f * nb, nb) < 0) bad = f;
    }
#endif
    PyMem_Free(rows);
    PyBuffer_Release(&oview);
    return PyLong_FromSsize_t(bad);
}

/* [None] * n, for f64_into_list to fill. */
static PyObject* none_list(PyObject* self, PyObject* args) {
    Py_ssize_t n;
    if (!PyArg_ParseTuple(args, "n", &n)) return NULL;
    if (n < 0) {
        PyErr_SetString(PyExc_ValueError, "negative length");
        return NULL;
    }
    return make_none_list(n);
}

/* n distinct float objects (0.0), each held by the returned list only: the aggregate's output made
 * ahead (SecaggCrypter.prepare_aggregate), whose values fill_slots then writes in place. */
static PyObject* float_pool(PyObject* self, PyObject* args) {
    Py_ssize_t n;
    if (!PyArg_ParseTuple(args, "n", &n)) return NULL;
    if (n < 0) {
        PyErr_SetString(PyExc_ValueError, "negative length");
        return NULL;
    }
    PyObject* lst = PyList_New(n);
    if (!lst) return NULL;
    PyObject** items = ((PyListObject*)lst)->ob_item;
    for (Py_ssize_t i = 0; i < n; ++i) {
        items[i] = PyFloat_FromDouble(0.0);
        if (!items[i]) {
            for (Py_ssize_t j = i; j < n; ++j) { /* the rest None: the list stays well-formed */
                Py_INCREF(Py_None);
                items[j] = Py_None;
            }
            Py_DECREF(lst);
            return NULL;
        }
    }
    return lst;
}

/* ---- the reference's additive-share draws, exactly (AdditiveSecret.split with reference_rng) ----------
 * The reference draws every share with the global `random` (`_additive_ss.py:96`: random.randint(0, 2**bl)
 * per element, per share, element-major), i.e. CPython's MT19937 (Matsumoto & Nishimura 1998, the 32-bit
 * generator with its tempering) behind randint -> randrange -> _randbelow_with_getrandbits(n = 2**bl + 1):
 * k = n.bit_length() bits per attempt, getrandbits(k) = 32-bit outputs least significant first with the
 * last one shifted right to its k mod 32 bits, rejected while >= n.  mt_share_draws runs that from the
 * state `random.getstate()` holds and returns the state `random.setstate()` takes back, so the Python
 * stream goes on where the reference's would. */
#define MT_N 624
#define MT_M 397

static uint32_t mt_next(uint32_t* mt, Py_ssize_t* idx) {
    if (*idx >= MT_N) {
        int kk;
        uint32_t y;
        for (kk = 0; kk < MT_N - MT_M; ++kk) {
            y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        for (; kk < MT_N - 1; ++kk) {
            y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
        mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        *idx = 0;
    }
    uint32_t y = mt[(*idx)++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* randint(0, 2**bl) for bl <= 126, as (lo, hi) of a non-negative int128 */
static void mt_randint_pow2(uint32_t* mt, Py_ssize_t* idx, int bl, uint64_t* lo, uint64_t* hi) {
    const int k = bl == 0 ? 2 : bl + 1; /* (2**bl + 1).bit_length() */
    for (;;) {
        uint32_t w[4] = {0, 0, 0, 0};
        int rem = k;
        for (int i = 0; rem > 0; ++i, rem -= 32) {
            uint32_t r = mt_next(mt, idx);
            if (rem < 32) r >>= 32 - rem;
            w[i] = r;
        }
        const uint64_t l = (uint64_t)w[0] | ((uint64_t)w[1] << 32), h = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
        const int accept = bl < 64 ? h == 0 && l <= (1ull << bl)  /* r <= 2**bl */
                                   : h < (1ull << (bl - 64)) || (h == (1ull << (bl - 64)) && l == 0);
        if (accept) {
            *lo = l;
            *hi = h;
            return;
        }
    }
}

static PyObject* mt_share_draws(PyObject* self, PyObject* args) {
    /* (state: 625-tuple of ints, bls: uint32 buffer [n], draws: int, out: int64 buffer [draws, n, 2])
     * -> the 625-tuple after the draws */
    PyObject *state, *out;
    Py_buffer bv, ov;
    Py_ssize_t reps;
    if (!PyArg_ParseTuple(args, "O!y*nO", &PyTuple_Type, &state, &bv, &reps, &out)) return NULL;
    if (PyTuple_GET_SIZE(state) != MT_N + 1 || bv.len % 4 || reps < 0) {
        PyBuffer_Release(&bv);
        PyErr_SetString(PyExc_ValueError, "mt_share_draws takes a 625-entry MT19937 state and uint32 bit lengths");
        return NULL;
    }
    const Py_ssize_t n = bv.len / 4;
    if (get_out(out, &ov, reps * n * 16) < 0) {
        PyBuffer_Release(&bv);
        return NULL;
    }
    uint32_t mt[MT_N];
    for (int i = 0; i < MT_N; ++i) mt[i] = (uint32_t)PyLong_AsUnsignedLongMask(PyTuple_GET_ITEM(state, i));
    Py_ssize_t idx = PyLong_AsSsize_t(PyTuple_GET_ITEM(state, MT_N));
    const uint32_t* bls = (const uint32_t*)bv.buf;
    uint64_t* o = (uint64_t*)ov.buf;
    int bad = PyErr_Occurred() != NULL || idx < 0 || idx > MT_N;
    for (Py_ssize_t i = 0; i < n && !bad; ++i) {
        if (bls[i] > 126) {
            bad = 1;
            break;
        }
        for (Py_ssize_t j = 0; j < reps; ++j) {
            uint64_t* d = o + 2 * (j * n + i);
            mt_randint_pow2(mt, &idx, (int)bls[i], d, d + 1);
        }
    }
    PyBuffer_Release(&bv);
    PyBuffer_Release(&ov);
    if (bad) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "bit length above 126 or a bad MT19937 index");
        return NULL;
    }
    PyObject* res = PyTuple_New(MT_N + 1);
    if (!res) return NULL;
    for (int i = 0; i < MT_N; ++i) {
        PyObject* v = PyLong_FromUnsignedLong(mt[i]);
        if (!v) {
            Py_DECREF(res);
            return NULL;
        }
        PyTuple_SET_ITEM(res, i, v);
    }
    PyObject* v = PyLong_FromSsize_t(idx);
    if (!v) {
        Py_DECREF(res);
        return NULL;
    }
    PyTuple_SET_ITEM(res, MT_N, v);
    return res;
}

/* all_ints over a list of lists in one call: every party's list at once, split evenly over host threads
 * (the researcher's type check of 8 x 333 334 ciphertexts: one thread pool instead of one per list) ->
 * -1, or the index of the first list holding an item that is not an int (isinstance semantics). */
typedef struct {
    PyObject* const* lists;
    const Py_ssize_t* start; /* start[u] = items before list u */
    Py_ssize_t n_lists, lo, hi;
    Py_ssize_t bad; /* the first bad list in [lo, hi), or -1 */
} intchk2_job;

static void* intchk2_range(void* arg) {
    intchk2_job* j = (intchk2_job*)arg;
    j->bad = -1;
    Py_ssize_t u = 0;
    while (u + 1 < j->n_lists && j->start[u + 1] <= j->lo) ++u;
    for (Py_ssize_t g = j->lo; g < j->hi; ++g) {
        while (g >= j->start[u + 1]) ++u;
        PyObject* v = ((PyListObject*)j->lists[u])->ob_item[g - j->start[u]];
        if (!PyLong_Check(v)) {
            j->bad = u;
            return NULL;
        }
    }
    return NULL;
}

static PyObject* all_ints_lists(PyObject* self, PyObject* args) {
    PyObject* outer;
    if (!PyArg_ParseTuple(args, "O!", &PyList_Type, &outer)) return NULL;
    const Py_ssize_t P = PyList_GET_SIZE(outer);
    PyObject* const* lists = ((PyListObject*)outer)->ob_item;
    Py_ssize_t* start = (Py_ssize_t*)malloc((size_t)(P + 1) * sizeof(Py_ssize_t));
    if (!start) return PyErr_NoMemory();
    start[0] = 0;
    for (Py_ssize_t u = 0; u < P; ++u) {
        if (!PyList_Check(lists[u])) {
            free(start);
            PyErr_SetString(PyExc_TypeError, "all_ints_lists takes a list of lists");
            return NULL;
        }
        start[u + 1] = start[u] + PyList_GET_SIZE(lists[u]);
    }
    const Py_ssize_t n = start[P];
    const int nt = n >= (1 << 16) ? conv_threads(n) : 1;
    intchk2_job jobs[64];
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (intchk2_job){lists, start, P, n * t / nt, n * (t + 1) / nt, -1};
        if (t > 0) started[t] = pthread_create(&tid[t], NULL, intchk2_range, &jobs[t]) == 0;
    }
    intchk2_range(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            intchk2_range(&jobs[t]);
    }
    Py_ssize_t bad = -1;
    for (int t = 0; t < nt && bad < 0; ++t) bad = jobs[t].bad;
    free(start);
    return PyLong_FromSsize_t(bad);
}

/* An output list of ints made ahead (prepare_encrypt): n ints allocated with room for the digits of an
 * nb-byte value and holding 0 (ob_size 0: no digit is read).  words_into_pool later writes each one's value
 * in place -- no allocation on the encrypt's critical path (making 333 334 ciphertext-sized ints is ~17 ms
 * of page faults and allocator work on one thread).  None where the digit layout is not this build's
 * (FBM_DIGITS_FAST=0). */
static PyObject* int_pool(PyObject* self, PyObject* args) {
    Py_ssize_t n, nb;
    if (!PyArg_ParseTuple(args, "nn", &n, &nb)) return NULL;
    if (n < 0 || nb <= 0 || nb % 4) {
        PyErr_SetString(PyExc_ValueError, "int_pool takes n >= 0 and a positive width in whole 32-bit words");
        return NULL;
    }
#if FBM_DIGITS_FAST && FBM_INPLACE
    const Py_ssize_t nd = (8 * nb + PyLong_SHIFT - 1) / PyLong_SHIFT;
    PyObject* lst = PyList_New(n);
    if (!lst) return NULL;
    PyObject** items = ((PyListObject*)lst)->ob_item;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyLongObject* v = _PyLong_New(nd);
        if (!v) {
            Py_DECREF(lst); /* the NULL slots after i are skipped by the list's deallocation */
            return NULL;
        }
        Py_SET_SIZE(v, 0);
        items[i] = (PyObject*)v;
    }
    return lst;
#else
    Py_RETURN_NONE;
#endif
}

#if FBM_DIGITS_FAST && FBM_INPLACE
typedef struct {
    PyObject** items;
    const unsigned char* src;
    Py_ssize_t lo, hi, nb;
} pool_job;

static void* pool_range(void* arg) {
    pool_job* j = (pool_job*)arg;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
        const uint32_t* w = (const uint32_t*)(j->src + i * j->nb);
        const Py_ssize_t nw = words_used(w, j->nb / 4);
        PyLongObject* v = (PyLongObject*)j->items[i];
        if (nw == 0) {
            Py_SET_SIZE(v, 0);
            continue;
        }
        const Py_ssize_t nbits = 32 * (nw - 1) + (32 - __builtin_clz(w[nw - 1]));
        Py_SET_SIZE(v, (nbits + PyLong_SHIFT - 1) / PyLong_SHIFT);
        long_fill(v, w, nw);
    }
    return NULL;
}
#endif

/* The values of buf (n x nb bytes, unsigned little-endian, nb the pool's width) into int_pool's ints
 * [off, off + n), in place, on host threads while this thread holds the GIL.  Every item must be an exact int that only the
 * list holds (refcount 1): the pool's own, never handed out -- anything else is a ValueError and nothing
 * is written. */
static PyObject* words_into_pool(PyObject* self, PyObject* args) {
    PyObject* lst;
    Py_buffer view;
    Py_ssize_t nb, off = 0;
    if (!PyArg_ParseTuple(args, "O!y*n|n", &PyList_Type, &lst, &view, &nb, &off)) return NULL;
#if FBM_DIGITS_FAST && FBM_INPLACE
    const Py_ssize_t n = nb > 0 ? view.len / nb : 0;
    if (nb <= 0 || nb % 4 || view.len % nb || ((uintptr_t)view.buf & 3) || off < 0 ||
        off + n > PyList_GET_SIZE(lst)) {
        PyBuffer_Release(&view);
        PyErr_SetString(PyExc_ValueError, "buffer does not hold whole 32-bit-word values for the pool at that offset");
        return NULL;
    }
    PyObject** items = ((PyListObject*)lst)->ob_item + off;
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (!PyLong_CheckExact(items[i]) || Py_REFCNT(items[i]) != 1) {
            PyBuffer_Release(&view);
            PyErr_SetString(PyExc_ValueError, "words_into_pool fills the ints of an int_pool that nothing else holds");
            return NULL;
        }
    }
    const int nt = n * nb >= PAR_MIN_BYTES ? conv_threads(n) : 1;
    pool_job jobs[64];
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (pool_job){items, (const unsigned char*)view.buf, n * t / nt, n * (t + 1) / nt, nb};
        if (t > 0) started[t] = pthread_create(&tid[t], NULL, pool_range, &jobs[t]) == 0;
    }
    pool_range(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            pool_range(&jobs[t]);
    }
    PyBuffer_Release(&view);
    Py_RETURN_NONE;
#else
    (void)lst, (void)nb, (void)off;
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "no int pools in this build (CPython other than 3.10 / 3.11, or FBM_INPLACE=0)");
    return NULL;
#endif
}

/* list[offset:offset + k] = the k float64 values of buf (one pass: no intermediate list as
 * ndarray.tolist() + extend would build), slot by slot as fill_slots says. */
/* A long f64_into_list on host threads WHILE THIS THREAD HOLDS THE GIL: a check pass (every slot None or an
 * exact float: the type pointers only), then the in-place writes of the floats nothing else holds (ob_fval
 * of objects only the list references -- a prepared pool's 10M floats: ~22 ms on one thread).  The slots
 * left (None, or a float with another holder: an allocation and a DECREF each) go through fill_slots on
 * this thread, which skips the floats already written. */
typedef struct {
    PyObject** items;
    const double* src;
    Py_ssize_t lo, hi, bad, rest;
} slot_job;

static void* slot_check_range(void* arg) {
    slot_job* j = (slot_job*)arg;
    j->bad = -1;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i)
        if (j->items[i] != Py_None && !PyFloat_CheckExact(j->items[i])) {
            j->bad = i;
            break;
        }
    return NULL;
}

static void* slot_fill_range(void* arg) {
    slot_job* j = (slot_job*)arg;
    j->rest = 0;
    for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
        PyObject* o = j->items[i];
        if (FBM_INPLACE && o != Py_None && Py_REFCNT(o) == 1)
            ((PyFloatObject*)o)->ob_fval = j->src[i];
        else
            ++j->rest;
    }
    return NULL;
}

static void run_slot_jobs(slot_job* jobs, int nt, void* (*fn)(void*)) {
    pthread_t tid[64];
    int started[64] = {0};
    for (int t = 1; t < nt; ++t) started[t] = pthread_create(&tid[t], NULL, fn, &jobs[t]) == 0;
    fn(&jobs[0]);
    for (int t = 1; t < nt; ++t) {
        if (started[t])
            pthread_join(tid[t], NULL);
        else
            fn(&jobs[t]);
    }
}

static int slots_parallel(PyObject** items, const double* src, Py_ssize_t k, int nt) {
    slot_job jobs[64];
    for (int t = 0; t < nt; ++t) jobs[t] = (slot_job){items, src, k * t / nt, k * (t + 1) / nt, -1, 0};
    run_slot_jobs(jobs, nt, slot_check_range);
    for (int t = 0; t < nt; ++t)
        if (jobs[t].bad >= 0) {
            PyErr_SetString(PyExc_ValueError, "f64_into_list fills slots that hold None or floats only");
            return -1;
        }
    run_slot_jobs(jobs, nt, slot_fill_range);
    Py_ssize_t rest = 0;
    for (int t = 0; t < nt; ++t) rest += jobs[t].rest;
    return rest ? fill_slots(items, src, k) : 0;
}

static PyObject* f64_into_list(PyObject* self, PyObject* args) {
    PyObject* lst;
    Py_ssize_t off;
    Py_buffer view;
    if (!PyArg_ParseTuple(args, "O!ny*", &PyList_Type, &lst, &off, &view)) return NULL;
    const Py_ssize_t k = view.len / (Py_ssize_t)sizeof(double);
    if (view.len % (Py_ssize_t)sizeof(double) || off < 0 || off + k > PyList_GET_SIZE(lst)) {
        PyBuffer_Release(&view);
        PyErr_SetString(PyExc_ValueError, "float64 buffer does not fit the list at that offset");
        return NULL;
    }
    const double* src = (const double*)view.buf;
    PyObject** items = ((PyListObject*)lst)->ob_item + off;
    /* threads for a pool's floats; a list of None (the unprepared aggregate's) allocates every slot here */
    const int nt = k >= (1 << 16) && items[0] != Py_None ? conv_threads(k) : 1;
    int rc;
    if (nt == 1) {
        rc = check_slots(items, k) < 0 ? -1 : fill_slots(items, src, k);
    } else {
        rc = slots_parallel(items, src, k, nt);
    }
    PyBuffer_Release(&view);
    if (rc < 0) return NULL;
    Py_RETURN_NONE;
}

/* Whether this build writes into objects it made ahead (FBM_INPLACE) and reads / builds ints digit by digit
 * (FBM_DIGITS_FAST): (inplace, digits). */
static PyObject* build_flags(PyObject* self, PyObject* args) {
    (void)self, (void)args;
    return Py_BuildValue("(ii)", FBM_INPLACE ? 1 : 0, FBM_DIGITS_FAST ? 1 : 0);
}

static PyMethodDef methods[] = {
    {"build_flags", build_flags, METH_NOARGS, "-> (in-place writes into pool objects, digit-level int paths)"},
    {"all_ints", all_ints, METH_VARARGS, "list -> all items are ints (isinstance)"},
    {"mt_share_draws", mt_share_draws, METH_VARARGS,
     "MT19937 state (625-tuple), uint32 bit lengths [n], draws, int64 out [draws, n, 2] -> the state after: "
     "random.randint(0, 2**bl) element-major, as the reference's AdditiveSecret.split draws"},
    {"all_ints_lists", all_ints_lists, METH_VARARGS,
     "list of lists -> -1, or the first list holding a non-int (isinstance)"},
    {"floats_to_f64", floats_to_f64, METH_VARARGS, "list of floats -> float64 buffer; -1 or first bad index"},
    {"ints_to_bytes", ints_to_bytes, METH_VARARGS, "list of ints -> n-byte LE unsigned; -1 or first bad index"},
    {"bytes_to_ints", bytes_to_ints, METH_VARARGS, "buffer of n-byte LE unsigned values -> list of ints"},
    {"none_list", none_list, METH_VARARGS, "n -> [None] * n"},
    {"set_conv_threads", set_conv_threads, METH_VARARGS,
     "default host-thread count of the threaded loops (FBM_CONV_THREADS overrides it) -> the previous one"},
    {"float_pool", float_pool, METH_VARARGS, "n -> n distinct 0.0 floats held by the list only"},
    {"int_pool", int_pool, METH_VARARGS, "n, nb -> n fresh ints with room for nb-byte values (None: not this build)"},
    {"words_into_pool", words_into_pool, METH_VARARGS,
     "int_pool list, buffer of n nb-byte LE values, nb[, offset] -> None (each int's value written in place)"},
    {"ints_to_bytes_held", ints_to_bytes_held, METH_VARARGS,
     "lists, lo, hi, n, out -> -1 or first bad flat index (host threads, GIL held, no pins)"},
    {"f64_into_list", f64_into_list, METH_VARARGS, "list, offset, float64 buffer -> None (fills the list)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fbm_pyconv", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fbm_pyconv(void) { return PyModule_Create(&module); }
