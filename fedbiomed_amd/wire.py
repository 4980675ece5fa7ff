"""Wire format for encrypted model updates.

The reference ships a JL update as a list of Python ints through its msgpack `Serializer`
(`fedbiomed/common/serializer.py:96-110`): every ciphertext >= 2^64 goes through
`Serializer._default` and becomes its own ``{"__type__": "int", "value": <big-endian
bytes>}`` map -- one Python call, one ``to_bytes`` and ~270 bytes of framing per ciphertext
(333 334 of them per party for a 10M-parameter model), and on the researcher one
``object_hook`` call + ``int.from_bytes`` each, then ``int.to_bytes`` again to reach the
device.  A LOM update (uint64 ints) packs natively, but still one msgpack item per element.

`EncryptedParams` is a ``list`` of the same Python ints the reference API returns, which
also carries the device's packed form (JL: ``[n_ct, 64]`` little-endian u32 limbs; LOM:
``[n]`` u64 words).  It is only returned by the crypters once `enable()` has been called --
by default they return plain lists, so an unmodified reference `Serializer` (msgpack with
``strict_types=True`` hands list subclasses to ``_default``, which would refuse them) keeps
working.  With it enabled:

* the maintainer adds two lines to `Serializer._default` / `_object_hook`
  (INTEGRATION.md §Wire format) calling `to_wire` / `from_wire`: one msgpack ``bin`` per
  update instead of one map per ciphertext;
* `SecaggCrypter.aggregate` / `SecaggLomCrypter.aggregate` take the packed form straight to
  the device when every row is an `EncryptedParams` (no ``int.to_bytes`` per ciphertext).

`from_wire` materialises the Python ints as well, so every consumer that treats the update as
``List[int]`` sees exactly the reference's values.

`ChunkAssembler` is the other half of §8(f)2: the gRPC transport streams a serialized message in
chunks of `MAX_MESSAGE_BYTES_LENGTH` (4 MB) and the receiver rebuilds it with ``reply += chunk``
(`fedbiomed/transport/server.py:236-239`, `client.py:599-602` in `_call_researcher`), which copies the growing message at
every chunk -- quadratic in the chunk count (a 10M-parameter JL update is 22-24 chunks).  The
assembler keeps the chunks and joins them once.
"""

from __future__ import annotations

from typing import Any, Dict, Iterable, Optional

import numpy as np

WIRE_TYPE = "fedbiomed_amd.EncryptedParams"
_ENABLED = False


def enable(on: bool = True) -> None:
    """Make the crypters return `EncryptedParams` (call once the Serializer hook is in)."""
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


class EncryptedParams(list):
    """A reference-compatible ``List[int]`` update plus its packed device form.

    scheme "jl": ``packed`` is uint32 ``[n_ct, 64]`` (ciphertext k = little-endian limbs);
    scheme "lom": ``packed`` is uint64 ``[n]``.
    """

    __slots__ = ("scheme", "packed")

    def __init__(self, values: Iterable[int], scheme: str, packed: np.ndarray):
        super().__init__(values)
        if scheme not in ("jl", "lom"):
            raise ValueError("scheme must be 'jl' or 'lom'")
        self.scheme = scheme
        self.packed = packed

    @classmethod
    def from_ints(cls, scheme: str, values) -> "EncryptedParams":
        """Pack a plain update (JL ciphertexts must lie in [0, 2^2048), LOM words in [0, 2^64))."""
        values = [int(v) for v in values]
        if scheme == "jl":
            blob = b"".join(v.to_bytes(256, "little") for v in values)
            packed = np.frombuffer(blob, dtype="<u4").reshape(len(values), 64).copy()
        else:
            packed = np.array(values, dtype=np.uint64)
        return cls(values, scheme, packed)

    @classmethod
    def from_packed(cls, scheme: str, packed: np.ndarray) -> "EncryptedParams":
        packed = np.ascontiguousarray(packed)
        if scheme == "jl":
            from . import _device as D  # (the C conversion module: the ints' digits written on host threads)

            packed = packed.view(np.uint32).reshape(-1, 64)
            values = D.limbs_to_ints(packed)
        else:
            packed = packed.view(np.uint64).reshape(-1)
            values = packed.tolist()
        return cls(values, scheme, packed)

    def _drop(self) -> None:
        self.packed = None  # mutated: the ints are the truth from now on

    def __setitem__(self, i, v):
        self._drop()
        super().__setitem__(i, v)

    def __delitem__(self, i):
        self._drop()
        super().__delitem__(i)

    def __iadd__(self, other):
        self._drop()
        return super().__iadd__(other)

    def __imul__(self, k):
        self._drop()
        return super().__imul__(k)

    def _mutator(name):  # noqa: N805 - class-body helper
        def f(self, *a, **k):
            self._drop()
            return getattr(list, name)(self, *a, **k)
        f.__name__ = name
        return f

    append = _mutator("append")
    extend = _mutator("extend")
    insert = _mutator("insert")
    pop = _mutator("pop")
    remove = _mutator("remove")
    clear = _mutator("clear")
    sort = _mutator("sort")
    reverse = _mutator("reverse")
    del _mutator

    def consistent(self) -> bool:
        """True while the packed form still mirrors the list (every mutating list method
        drops it; the aggregate then converts the ints like a plain list)."""
        return self.packed is not None and self.packed.shape[0] == len(self)

    def to_wire(self) -> Dict[str, Any]:
        """The Serializer-hook form: one msgpack map holding one bin."""
        if not self.consistent():  # mutated: re-pack from the ints
            self.packed = (EncryptedParams.from_ints(self.scheme, list(self)).packed)
        return {"__type__": WIRE_TYPE, "value": [self.scheme, self.packed.dtype.str, list(self.packed.shape),
                                                 self.packed.tobytes()]}


def to_wire(obj: Any) -> Optional[Dict[str, Any]]:
    """For `Serializer._default`: the wire map of an `EncryptedParams`, else None."""
    return obj.to_wire() if isinstance(obj, EncryptedParams) else None


def from_wire(obj: Any) -> Any:
    """For `Serializer._object_hook`: rebuild an `EncryptedParams` from its wire map
    (anything else is returned unchanged)."""
    if isinstance(obj, dict) and obj.get("__type__") == WIRE_TYPE:
        scheme, dtype, shape, data = obj["value"]
        if scheme not in ("jl", "lom") or np.dtype(dtype) not in (np.dtype("<u4"), np.dtype("<u8")):
            raise ValueError("malformed EncryptedParams wire map")
        arr = np.frombuffer(data, dtype=np.dtype(dtype)).reshape(shape).copy()
        return EncryptedParams.from_packed(scheme, arr)
    return obj


def packed_rows(params, scheme: str, n: Optional[int] = None) -> Optional[np.ndarray]:
    """The stacked packed form of an aggregate's rows when every row is a consistent
    `EncryptedParams` of `scheme` (first `n` entries of each), else None."""
    if not params or not all(isinstance(p, EncryptedParams) and p.scheme == scheme for p in params):
        return None
    if not all(p.consistent() for p in params):
        return None
    if n is None:  # LOM: rows must agree in length (the reference's np.array raises otherwise)
        if len({len(p) for p in params}) != 1:
            return None
        n = len(params[0])
    return np.stack([p.packed[:n] for p in params])


class ChunkAssembler:
    """Rebuilds a message streamed as chunks numbered ``iteration`` = 1 .. ``size`` (the transport's
    `TaskResult` / `TaskResponse` fields) in linear time.  ``add`` returns the whole message on its last
    chunk (``iteration == size``, the reference's completion test) and None before; the assembler is
    then empty for the next message, as the reference's loop is after ``Serializer.loads``."""

    __slots__ = ("_parts",)

    def __init__(self) -> None:
        self._parts: list = []

    def add(self, chunk: bytes, size: int, iteration: int) -> Optional[bytes]:
        self._parts.append(chunk)
        if size != iteration:
            return None
        out = b"".join(self._parts)
        self._parts = []
        return out
