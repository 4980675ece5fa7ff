"""Minimal stand-in for the `gmpy2` module, used ONLY to import the reference
Fed-BioMed crypter in the survey container (gmpy2 is not installed and there is
no network).  It is test tooling for `tools/gen_golden.py`; nothing under
`fedbiomed_amd/` imports it.

Semantics follow gmpy2 2.1.5 (pinned in the reference's pdm.lock) for the
subset the reference hot path touches (`_jls.py:30-73,289-374,702-762`):

* `mpz` is a separate class (NOT an `int` subclass) so that numpy builds
  object arrays from lists of mpz exactly as with the real gmpy2.
* `powmod` goes to the system GMP (`libgmp.so.10`, `__gmpz_powm`) through
  ctypes, i.e. the very library gmpy2 wraps; negative exponents invert first.
"""

import ctypes
import ctypes.util
import math
import numbers

_gmp = ctypes.CDLL(ctypes.util.find_library("gmp") or "libgmp.so.10")


class _MpzStruct(ctypes.Structure):
    _fields_ = [("alloc", ctypes.c_int), ("size", ctypes.c_int), ("d", ctypes.c_void_p)]


_P = ctypes.POINTER(_MpzStruct)
_gmp.__gmpz_init.argtypes = [_P]
_gmp.__gmpz_clear.argtypes = [_P]
_gmp.__gmpz_import.argtypes = [_P, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t,
                               ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
_gmp.__gmpz_export.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                               ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t, _P]
_gmp.__gmpz_export.restype = ctypes.c_void_p
_gmp.__gmpz_powm.argtypes = [_P, _P, _P, _P]


def _to_gmp(z: _MpzStruct, v: int) -> None:
    assert v >= 0
    nbytes = max(1, (v.bit_length() + 7) // 8)
    buf = v.to_bytes(nbytes, "big")
    _gmp.__gmpz_import(ctypes.byref(z), nbytes, 1, 1, 1, 0, buf)


def _from_gmp(z: _MpzStruct) -> int:
    nbytes = (abs(z.size) * 64 + 7) // 8 + 1
    buf = ctypes.create_string_buffer(nbytes)
    count = ctypes.c_size_t(0)
    _gmp.__gmpz_export(buf, ctypes.byref(count), 1, 1, 1, 0, ctypes.byref(z))
    return int.from_bytes(buf.raw[: count.value], "big")


def _gmp_powm(b: int, e: int, m: int) -> int:
    zs = [_MpzStruct() for _ in range(4)]
    for z in zs:
        _gmp.__gmpz_init(ctypes.byref(z))
    try:
        _to_gmp(zs[1], b)
        _to_gmp(zs[2], e)
        _to_gmp(zs[3], m)
        _gmp.__gmpz_powm(ctypes.byref(zs[0]), ctypes.byref(zs[1]), ctypes.byref(zs[2]), ctypes.byref(zs[3]))
        return _from_gmp(zs[0])
    finally:
        for z in zs:
            _gmp.__gmpz_clear(ctypes.byref(z))


def _i(o):
    if isinstance(o, mpz):
        return o._v
    if isinstance(o, (int, numbers.Integral)) and not isinstance(o, bool):
        return int(o)
    if isinstance(o, bool):
        return int(o)
    return None


class mpz:  # noqa: N801 - mirrors gmpy2's name
    __slots__ = ("_v",)

    def __init__(self, v=0, base=10):
        if isinstance(v, mpz):
            self._v = v._v
        elif isinstance(v, str):
            self._v = int(v, base)
        elif isinstance(v, float):
            self._v = int(v)
        else:
            self._v = int(v)

    # conversions
    def __int__(self):
        return self._v

    def __index__(self):
        return self._v

    def __float__(self):
        return float(self._v)

    def __bool__(self):
        return self._v != 0

    def __hash__(self):
        return hash(self._v)

    def __repr__(self):
        return f"mpz({self._v})"

    def __str__(self):
        return str(self._v)

    def digits(self, base=10):
        if base == 10:
            return str(self._v)
        if base == 16:
            return format(self._v, "x")
        if base == 2:
            return format(self._v, "b")
        raise ValueError("unsupported base")

    def bit_length(self):
        return self._v.bit_length()

    # arithmetic helpers
    def _bin(op):  # noqa: N805
        def f(self, o):
            x = _i(o)
            if x is None:
                return NotImplemented
            return mpz(op(self._v, x))

        def r(self, o):
            x = _i(o)
            if x is None:
                return NotImplemented
            return mpz(op(x, self._v))

        return f, r

    __add__, __radd__ = _bin(lambda a, b: a + b)
    __sub__, __rsub__ = _bin(lambda a, b: a - b)
    __mul__, __rmul__ = _bin(lambda a, b: a * b)
    __floordiv__, __rfloordiv__ = _bin(lambda a, b: a // b)
    __mod__, __rmod__ = _bin(lambda a, b: a % b)
    __lshift__, __rlshift__ = _bin(lambda a, b: a << b)
    __rshift__, __rrshift__ = _bin(lambda a, b: a >> b)
    __and__, __rand__ = _bin(lambda a, b: a & b)
    __or__, __ror__ = _bin(lambda a, b: a | b)
    __xor__, __rxor__ = _bin(lambda a, b: a ^ b)
    del _bin

    def __truediv__(self, o):
        x = _i(o)
        if x is None:
            return NotImplemented
        return self._v / x

    def __pow__(self, e, m=None):
        x = _i(e)
        if x is None:
            return NotImplemented
        if m is None:
            return mpz(self._v ** x)
        return powmod(self, x, m)

    def __neg__(self):
        return mpz(-self._v)

    def __pos__(self):
        return self

    def __abs__(self):
        return mpz(abs(self._v))

    def _cmp(op):  # noqa: N805
        def f(self, o):
            x = _i(o)
            if x is None:
                if isinstance(o, float):
                    return op(self._v, o)
                return NotImplemented
            return op(self._v, x)

        return f

    __eq__ = _cmp(lambda a, b: a == b)
    __ne__ = _cmp(lambda a, b: a != b)
    __lt__ = _cmp(lambda a, b: a < b)
    __le__ = _cmp(lambda a, b: a <= b)
    __gt__ = _cmp(lambda a, b: a > b)
    __ge__ = _cmp(lambda a, b: a >= b)
    del _cmp


def powmod(a, b, c):
    a, b, c = _i(a), _i(b), _i(c)
    if b < 0:
        a = pow(a, -1, c)  # raises ValueError if not invertible (gmpy2: ZeroDivisionError-like)
        b = -b
    return mpz(_gmp_powm(a % c, b, c))


def invert(a, b):
    a, b = _i(a), _i(b)
    try:
        return mpz(pow(a, -1, b))
    except ValueError as e:
        raise ZeroDivisionError("invert() no inverse exists") from e


def gcd(a, b):
    return mpz(math.gcd(_i(a), _i(b)))
