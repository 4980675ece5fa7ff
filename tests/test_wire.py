"""Wire format: EncryptedParams through a msgpack Serializer set up the way the
reference's is (`fedbiomed/common/serializer.py`: strict_types=True, big ints as
{"__type__": "int", "value": signed big-endian bytes}) with and without the two-line hook."""

import math

import msgpack
import numpy as np
import pytest

from fedbiomed_amd import wire


def _ref_default(obj):
    """The reference's big-int rule (serializer.py:103-110) -- the per-ciphertext cost."""
    if isinstance(obj, int):
        return {"__type__": "int", "value": obj.to_bytes(length=math.ceil(obj.bit_length() / 8) + 1,
                                                         byteorder="big", signed=True)}
    raise TypeError(f"Cannot serialize object of type '{type(obj)}'.")


def _ref_hook(obj):
    if isinstance(obj, dict) and obj.get("__type__") == "int":
        return int.from_bytes(obj["value"], byteorder="big", signed=True)
    return obj


def _hooked_default(obj):
    w = wire.to_wire(obj)
    return w if w is not None else _ref_default(obj)


def _hooked_hook(obj):
    return _ref_hook(wire.from_wire(obj))


def _dumps(obj, default):
    return msgpack.packb(obj, default=default, strict_types=True)


def _loads(b, hook):
    return msgpack.unpackb(b, object_hook=hook, strict_map_key=False)


def _jl_update(n_ct, seed=0):
    rng = np.random.default_rng(seed)
    limbs = rng.integers(0, 2**32, size=(n_ct, 64), dtype=np.uint64).astype(np.uint32)
    limbs[:, 63] >>= 1  # < 2^2047
    return wire.EncryptedParams.from_packed("jl", limbs)


def test_plain_list_semantics():
    e = _jl_update(50)
    assert isinstance(e, list) and all(isinstance(v, int) for v in e)
    assert e == list(e) and e.consistent()
    assert wire.EncryptedParams.from_ints("jl", list(e)).packed.tobytes() == e.packed.tobytes()
    lom = wire.EncryptedParams.from_ints("lom", [0, 1, 2**64 - 1])
    assert lom == [0, 1, 2**64 - 1] and lom.packed.dtype == np.uint64


def test_unhooked_serializer_refuses_the_subclass():
    """Why the crypters return EncryptedParams only after wire.enable(): msgpack with
    strict_types=True hands list subclasses to `default`, which the reference refuses."""
    with pytest.raises(TypeError):
        _dumps({"params": _jl_update(3)}, _ref_default)
    assert not wire.enabled()


@pytest.mark.parametrize("scheme", ["jl", "lom"])
def test_hooked_roundtrip_and_size(scheme):
    if scheme == "jl":
        e = _jl_update(400, seed=1)
    else:
        e = wire.EncryptedParams.from_ints("lom", np.random.default_rng(2).integers(0, 2**63, 5000).tolist())
    msg = {"researcher_id": "r", "params": e, "round": 3}
    blob = _dumps(msg, _hooked_default)
    back = _loads(blob, _hooked_hook)
    assert back["round"] == 3 and back["params"] == list(e)
    assert isinstance(back["params"], wire.EncryptedParams) and back["params"].consistent()
    assert np.array_equal(back["params"].packed, e.packed)
    # the reference encoding of the same plain list decodes to the same ints
    ref = _dumps({"researcher_id": "r", "params": list(e), "round": 3}, _ref_default)
    assert _loads(ref, _ref_hook)["params"] == back["params"]
    if scheme == "jl":  # one bin instead of one map per ciphertext
        assert len(blob) < 0.97 * len(ref)


def test_mutation_drops_the_packed_form():
    e = _jl_update(5)
    e[2] = 7
    assert not e.consistent()
    assert wire.packed_rows([e], "jl", 5) is None
    back = _loads(_dumps(e, _hooked_default), _hooked_hook)  # re-packed from the ints
    assert back == e and back.consistent()
    f = _jl_update(5)
    f.append(3)
    assert not f.consistent()


def test_packed_rows_rules():
    a, b = _jl_update(6, 1), _jl_update(4, 2)
    rows = wire.packed_rows([a, b], "jl", 4)
    assert rows.shape == (2, 4, 64)
    assert wire.packed_rows([a, list(b)], "jl", 4) is None  # one plain row: ints path
    la = wire.EncryptedParams.from_ints("lom", [1, 2, 3])
    lb = wire.EncryptedParams.from_ints("lom", [1, 2])
    assert wire.packed_rows([la, lb], "lom") is None  # ragged LOM: the reference's np.array error path
    assert wire.packed_rows([la, la], "lom").shape == (2, 3)


def test_malformed_wire_map():
    with pytest.raises(ValueError):
        wire.from_wire({"__type__": wire.WIRE_TYPE, "value": ["jl", "<f8", [1], b"\0" * 8]})


@pytest.mark.gpu
def test_crypters_through_the_wire():
    """encrypt (wire enabled) -> hooked dumps/loads -> aggregate takes the packed rows to the
    device; results equal the plain-list path bit for bit."""
    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    D.device()
    P, n, tau = 3, 2000, 2
    ws = [W.party_weight(p) for p in range(P)]
    xs = [W.party_params(p, n).astype(np.float64).tolist() for p in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    ids = W.node_ids(P)
    jc, lc = SecaggCrypter(), SecaggLomCrypter(W.LOM_NONCE)
    try:
        plain_j = [jc.encrypt(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
        plain_l = [lc.encrypt(tau, u, xs[p], W.pairwise_secrets_for(u, ids), ids, weight=ws[p])
                   for p, u in enumerate(ids)]
        assert type(plain_j[0]) is list and type(plain_l[0]) is list
        wire.enable()
        enc_j = [jc.encrypt(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
        enc_l = [lc.encrypt(tau, u, xs[p], W.pairwise_secrets_for(u, ids), ids, weight=ws[p])
                 for p, u in enumerate(ids)]
    finally:
        wire.enable(False)
    assert enc_j == plain_j and enc_l == plain_l
    recv_j = [_loads(_dumps(e, _hooked_default), _hooked_hook) for e in enc_j]
    recv_l = [_loads(_dumps(e, _hooked_default), _hooked_hook) for e in enc_l]
    assert wire.packed_rows(recv_j, "jl", len(recv_j[0])) is not None
    a = jc.aggregate(tau, P, recv_j, -sum(keys), W.BIPRIME0, sum(ws), num_expected_params=n)
    b = jc.aggregate(tau, P, plain_j, -sum(keys), W.BIPRIME0, sum(ws), num_expected_params=n)
    assert np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))
    a = lc.aggregate(recv_l, sum(ws))
    b = lc.aggregate(plain_l, sum(ws))
    assert np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


def test_chunk_assembler_matches_the_reference_loop():
    """ChunkAssembler returns the bytes the reference's ``reply += answer.bytes_`` loop builds
    (transport/server.py:236-239): one message per ``size == iteration`` chunk, several messages on one
    stream, chunk sizes as the sender cuts them (MAX_MESSAGE_BYTES_LENGTH, the last one short), a
    one-chunk message and an empty one."""
    import os as _os

    from fedbiomed_amd.wire import ChunkAssembler

    cut = 4000000 - 33  # the reference's MAX_MESSAGE_BYTES_LENGTH (constants.py:121)
    msgs = [_os.urandom(3 * cut + 12345), b"x" * 17, b"", _os.urandom(cut)]
    stream = []
    for m in msgs:
        starts = list(range(0, len(m), cut)) or [0]
        for it, st in enumerate(starts, 1):
            stream.append((m[st:st + cut], len(starts), it))
    asm, got, ref, reply = ChunkAssembler(), [], [], bytes()
    for chunk, size, it in stream:
        out = asm.add(chunk, size, it)
        if out is not None:
            got.append(out)
        reply += chunk  # the reference's loop
        if size == it:
            ref.append(reply)
            reply = bytes()
    assert got == ref == msgs
