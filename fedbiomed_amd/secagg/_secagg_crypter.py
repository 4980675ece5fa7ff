"""Drop-in secure-aggregation crypters backed by the MI355X HIP kernels.

Mirrors the reference boundary `fedbiomed/common/secagg/_secagg_crypter.py`:
  SecaggCrypter.encrypt     (:45-137)   SecaggCrypter.aggregate     (:139-230)
  SecaggLomCrypter.__init__ (:303-316)  SecaggLomCrypter.encrypt    (:318-392)
  SecaggLomCrypter.aggregate(:394-455)  _apply_average (:233-249)   _apply_weighting (:252-276)
Same signatures, same argument validation, same exceptions and messages; the arithmetic
(quantise, weight, PRF masks / VES pack + FDH + 2048-bit modexp, sums, unmask, average,
dequantise) runs on the GPU through `fedbiomed_amd._device` -> `include/fbm_secagg.h`.

Besides the list API, `encrypt_tensor` / `aggregate_tensor` take device tensors directly
(the fast path for callers that already hold the flattened model in HBM).
"""

from __future__ import annotations

import logging
import secrets
import time
from typing import Dict, List, Optional, Union

import numpy as np
import torch

from .. import _device as D, wire
from ..constants import ErrorNumbers, SAParameters
from ..exceptions import FedbiomedSecaggCrypterError
from ._jls import FDH, EncryptedNumber, PublicParam

logger = logging.getLogger("fedbiomed_amd")


def _check_weight(weight: Optional[int], jl: bool) -> None:
    """The reference's only weight check (`_secagg_crypter.py:106-111` JL, `:367-372` LOM): the
    bit length.  A negative weight passes it, as in the reference: JL then encrypts the
    negative packing (`_jls.py:169-176`, reproduced on the device), LOM raises numpy's
    OverflowError from its uint64 conversion (`_lom.py:153`, see SecaggLomCrypter)."""
    if weight is None:
        return
    if 2 ** weight.bit_length() > SAParameters.WEIGHT_RANGE:
        if jl:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: The weight is too large. The weight should be less than "
                f"{SAParameters.WEIGHT_RANGE}, but got {weight}")
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: The weight is too large. The weight should be less than "
            f"{SAParameters.WEIGHT_RANGE}.")


def _check_float_list(params) -> torch.Tensor:
    """The reference's list/float checks; returns the float64 host copy made in the same pass."""
    if not isinstance(params, list):
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: Expected argument `params` type list but got {type(params)}")
    host = D.floats_to_host(params)
    if host is None:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: The parameters to encrypt should list of floats. "
            f"There are one or more than a value that is not type of float.")
    return host


def _check_int_lists(params) -> None:
    if not isinstance(params, list) or not all(isinstance(p, list) for p in params):
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: The parameters to aggregate should be a "
            f"list containing list of parameters")
    if not D.all_ints_lists(params):
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: Invalid parameter type. The parameters "
            f"should be of type of integers.")


def _prep_tag(current_round, num_nodes, key, biprime, target_range) -> Optional[bytes]:
    """What prepare_aggregate's factors belong to, without keeping the key: SHA-256 over the arguments'
    length-prefixed two's-complement bytes (None when one is not an int: nothing matches it)."""
    import hashlib

    vals = (current_round, num_nodes, key, biprime, target_range or SAParameters.TARGET_RANGE)
    if not all(isinstance(v, int) for v in vals):
        return None
    h = hashlib.sha256()
    for v in vals:
        b = v.to_bytes(v.bit_length() // 8 + 1, "little", signed=True)
        h.update(len(b).to_bytes(8, "little") + b)
    return h.digest()


def _scrub_prep(prep, keys) -> None:
    """Zeroes a dropped preparation's factor tensors in HBM, on the current stream once their
    exponentiations (on the preparation's side stream) are done; the memory then returns to torch's
    caching allocator only after the zeroing."""
    if not prep:
        return
    ev = prep.get("event")
    for k in keys:
        v = prep.get(k)
        for t in (v if isinstance(v, list) else [v]):
            if t is None:
                continue
            st = torch.cuda.current_stream(t.device)
            if ev is not None:
                st.wait_event(ev)
            t.record_stream(st)
            t.zero_()


class SecaggCrypter:
    """Joye-Libert secure aggregation (encrypt on nodes, aggregate on the researcher)."""

    # prepare_encrypt's factor, held by the class: the node makes a SecaggCrypter per encrypt call
    # (`node/secagg/_secagg_round.py:139-157`), so the call that takes it is another instance's
    _enc_prep = None

    @staticmethod
    def _setup_public_param(biprime: int) -> PublicParam:
        """reference _secagg_crypter.py:28-43: N = biprime, bits 1024, FDH(2048, N^2).H (the
        object API's PublicParam; encrypt/aggregate themselves take the biprime directly)."""
        key_size = SAParameters.KEY_SIZE
        biprime = int(biprime)
        fdh = FDH(bits_size=key_size, n_modulus=biprime * biprime)
        return PublicParam(n_modulus=biprime, bits=key_size // 2, hashing_function=fdh.H)

    @staticmethod
    def _convert_to_encrypted_number(params: List[List[int]], public_param: PublicParam) -> List[List[EncryptedNumber]]:
        """reference _secagg_crypter.py:279-297"""
        return [[EncryptedNumber(public_param, int(param)) for param in parameters] for parameters in params]

    # ---- device fast path ------------------------------------------------------------------
    def encrypt_tensor(self, num_nodes: int, current_round: int, params: torch.Tensor, key: int, biprime: int,
                       clipping_range: Union[int, None] = None, weight: Optional[int] = None,
                       target_range: Optional[int] = None, ct_offset: int = 0, defer_exp: bool = False,
                       out: Optional[torch.Tensor] = None, factor: Optional[torch.Tensor] = None):
        """Device tensor (f32/f64) in HBM -> int32 [n_ct, 64] ciphertext limbs in HBM.
        `factor`: this party's H(t_k)^key of these ciphertexts computed ahead (`decrypt_factor_tensor` with
        the party's key, round and ct_offset; `prepare_encrypt` issues it for the list API): the encrypt is
        then one product per ciphertext instead of an exponentiation, with the same ciphertexts.
        `ct_offset`: global index of this shard's first ciphertext (element-range sharding).
        `out`: an int32 [n_ct, 64] destination (e.g. this party's row of the [P, n_ct, 64] block
        aggregate_tensor takes), as SecaggLomCrypter.encrypt_tensor's.
        `defer_exp`: issue the prologue kernels only and return a PendingEncrypt whose
        finish() issues the exponentiation (several parties on one device: every prologue
        before the first exponentiation occupies the chip)."""
        if not isinstance(key, int):
            raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: The argument `key` must be integer")
        target_range = target_range or SAParameters.TARGET_RANGE
        _check_weight(weight, jl=True)
        try:
            return D.jl_encrypt(params, biprime, key, current_round, num_nodes, clip=clipping_range,
                                target=target_range, weight=1 if weight is None else weight, ct_offset=ct_offset,
                                defer_exp=defer_exp, out=out, factor=factor)
        except (TypeError, ValueError) as exp:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value} Error during parameter encryption. {exp}") from exp

    def aggregate_tensor(self, current_round: int, cts: torch.Tensor, key: int, biprime: int,
                         total_sample_size: int, clipping_range: Union[int, None] = None,
                         num_expected_params: int = 1, target_range: Optional[int] = None,
                         want_sums: bool = False, ct_offset: int = 0,
                         decrypt_factor: Optional[torch.Tensor] = None):
        """[P, n_ct, 64] int32 ciphertext limbs in HBM -> float64 [n] averaged parameters.
        `decrypt_factor`: this round's `decrypt_factor_tensor` (computed ahead, e.g. while the
        nodes encrypt), or None to compute it here."""
        if not isinstance(key, int):
            raise TypeError("The key should be type of integer")
        target_range = target_range or SAParameters.TARGET_RANGE
        out, sums = D.jl_aggregate(cts, biprime, key, current_round, num_expected_params, total_sample_size,
                                   clip=clipping_range, target=target_range, want_sums=want_sums,
                                   ct_offset=ct_offset, factor=decrypt_factor)
        return (out, sums) if want_sums else out

    def decrypt_factor_tensor(self, current_round: int, num_ciphertexts: int, key: int, biprime: int,
                              ct_offset: int = 0, phased: bool = False):
        """The server key's per-ciphertext factor H(t_k)^key mod N^2 of round `current_round`
        (int32 [num_ciphertexts, 64] in HBM).  It does not depend on the parties' ciphertexts,
        so the researcher can compute it before they arrive and pass it to aggregate_tensor.
        `phased`: issue constants + FDH only and return a PendingFactor (exponentiate(),
        finish() -> tensor) so a caller can order its kernels against other work."""
        if not isinstance(key, int):
            raise TypeError("The key should be type of integer")
        return D.jl_decrypt_factor(num_ciphertexts, biprime, key, current_round, ct_offset=ct_offset,
                                   phased=phased)

    # ---- reference API -----------------------------------------------------------------------
    def encrypt(self, num_nodes: int, current_round: int, params: List[float], key: int, biprime: int,
                clipping_range: Union[int, None] = None, weight: Optional[int] = None,
                target_range: Optional[int] = None) -> List[int]:
        """Encrypts model parameters (reference `_secagg_crypter.py:45-137`).  If it raises, a
        prepare_encrypt preparation is dropped (drop_prepared)."""
        try:
            return self._encrypt(num_nodes, current_round, params, key, biprime, clipping_range, weight, target_range)
        except BaseException:
            SecaggCrypter.drop_prepared()
            raise

    def _encrypt(self, num_nodes, current_round, params, key, biprime, clipping_range, weight, target_range):
        start = time.process_time()
        host = _check_float_list(params)
        if not isinstance(key, int):
            raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: The argument `key` must be integer")
        target_range = target_range or SAParameters.TARGET_RANGE
        if params:  # quantize() evaluates nothing on an empty list, so it raises nothing there
            D.quant_params(clipping_range, target_range)  # OverflowError / range checks as the reference
        _check_weight(weight, jl=True)  # after quantize, before the (empty) protect: the reference's order
        if not params:
            return []
        try:  # the reference derives the slot inside jls.protect, under its try/except (:119-129)
            _, cr = D.jl_slot(target_range, num_nodes)
        except (TypeError, ValueError) as exp:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value} Error during parameter encryption. {exp}") from exp
        dev = D.device()
        x = host.to(dev, non_blocking=True)  # stream-ordered before the encrypt's kernels
        n_ct = (x.numel() + cr - 1) // cr
        prep = self._take_prepared_encrypt(current_round, num_nodes, key, biprime, target_range, n_ct, dev)
        if prep is not None:  # prepare_encrypt's factor: one product per ciphertext, no exponentiation
            factor, pool = prep
            ct = self.encrypt_tensor(num_nodes, current_round, x, key, biprime, clipping_range, weight, target_range,
                                     factor=factor)
            packed = D.to_host(ct).numpy().view(np.uint32)
            out = D.limbs_into_pool(pool, packed) if pool is not None else D.limbs_to_ints(packed)
        else:
            stripes = D.list_encrypt_stripes(n_ct, dev)
            if len(stripes) == 1:
                with D.deferred_checks():  # (checked at the exit, once the ciphertexts are back)
                    ct = self.encrypt_tensor(num_nodes, current_round, x, key, biprime, clipping_range, weight,
                                             target_range)
                    pool = D.int_pool(n_ct, prepared=False)  # the output's ints, made while the GPU exponentiates
                    packed = D.to_host(ct).numpy().view(np.uint32)
                out = D.limbs_into_pool(pool, packed, strict=True) if pool is not None else D.limbs_to_ints(packed)
            else:
                packed, out = self._encrypt_overlapped(num_nodes, current_round, x, key, biprime, clipping_range,
                                                       weight, target_range, stripes, cr)
        if wire.enabled():
            out = wire.EncryptedParams(out, "jl", packed)
        logger.debug(f"Encryption of the parameters took {time.process_time() - start} seconds.")
        return out

    def _encrypt_overlapped(self, num_nodes, current_round, x, key, biprime, clipping_range, weight, target_range,
                            stripes, cr):
        """The list API's encrypt as ct_offset stripes (one per full one-lane round, the partial round
        last), issued back to back on the current stream; each stripe's ciphertexts go to a pinned host
        buffer in stream order, right behind its kernels.  While the GPU exponentiates stripe 0 the host
        makes the output's int objects (`int_pool`), then writes stripe k's values into them while the GPU
        exponentiates stripe k + 1 (the ciphertext of index k depends only on k: the stripes concatenate
        bit for bit to the unsplit call's).  One status check for the whole call (its clipping warning
        once)."""
        dev, n = x.device, x.numel()
        host = D.host_empty((stripes[-1][1], 64), torch.int32)
        packed = host.numpy().view(np.uint32)
        main = torch.cuda.current_stream(dev)
        done = []
        with D.deferred_checks(merge=True):
            for c0, c1 in stripes:
                ct = self.encrypt_tensor(num_nodes, current_round, x[c0 * cr:min(n, c1 * cr)], key, biprime,
                                         clipping_range, weight, target_range, ct_offset=c0)
                # (in stream order: a side stream for the copies measured the same, 152-154 ms at 10M --
                # profiles/archive/r4_node_encrypt_probe.jsonl)
                host[c0:c1].copy_(ct, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(main)
                done.append(ev)
            pool = D.int_pool(stripes[-1][1], prepared=False)  # made while the GPU exponentiates stripe 0
            out = pool if pool is not None else []
            for (c0, c1), ev in zip(stripes, done):
                ev.synchronize()
                if pool is not None:
                    D.limbs_into_pool(pool, packed[c0:c1], c0, strict=True)
                else:
                    out += D.limbs_to_ints(packed[c0:c1])
        return packed, out

    def prepare_encrypt(self, current_round: int, num_nodes: int, key: int, biprime: int, num_params: int,
                        target_range: Optional[int] = None) -> bool:
        """Extension (not in the reference): issue a coming `encrypt`'s exponentiations now.  A node's
        ciphertext is c_k = (N pt_k + 1) H(t_k)^key mod N^2 (UserKey.encrypt, `_jls.py:473-505`); the
        factor H(t_k)^key depends only on the round, the node's key, the biprime and the vector's size,
        all known when the training request arrives (`node/secagg/_secagg_round.py`), so it can run on
        a side stream while the node trains.  The next `encrypt` of the same round, node count, key,
        biprime, target range and ciphertext count takes it (once) and only multiplies: the same
        ciphertexts, bit for bit.  Other calls of that round leave it, a call of another round drops
        it; a device condition of the early work is raised by the encrypt that takes it.  It also warms
        the encrypt's pinned staging buffers and makes its output list's int objects, whose values the
        encrypt writes in place (making 333 334 ciphertext-sized ints is ~17 ms).  Best effort: False
        (nothing prepared) where the encrypt would refuse the arguments, for an even N or N = 1, or with a
        library older than ABI 5.  The
        key itself is not kept, only a SHA-256 tag of it.  The preparation is the class's, not this
        instance's (one at a time): the node's encrypt runs on a fresh SecaggCrypter."""
        SecaggCrypter.drop_prepared()
        try:
            if not all(isinstance(v, int) for v in (current_round, num_nodes, key, biprime, num_params)):
                return False
            if num_nodes < 1 or biprime < 3 or biprime % 2 == 0:
                return False
            _, cr = D.jl_slot(target_range or SAParameters.TARGET_RANGE, num_nodes)
            n_ct = -(-num_params // cr)
            if n_ct <= 0:
                return False
            dev = D.device()
            from .. import _native as N

            if (N.loaded_abi or 0) < 5:
                return False
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side), D.capture_checks() as checks:
                factor = self.decrypt_factor_tensor(current_round, n_ct, key, biprime)
            ev = torch.cuda.Event()
            ev.record(side)
            warm = [D.host_empty((num_params,), torch.float64), D.host_empty((n_ct, 64), torch.int32)]
            del warm
            # and its output list: the int objects made now, their values written in place by the encrypt
            # (~300 B each: 100 MB at 10M elements, held until used or dropped)
            pool = D.int_pool(n_ct)
        except Exception:  # noqa: BLE001 -- encrypt raises whatever it is, in the reference's order
            return False
        SecaggCrypter._enc_prep = {"round": current_round,
                                   "tag": _prep_tag(current_round, num_nodes, key, biprime, target_range),
                                   "n_ct": n_ct, "factor": factor, "pool": pool, "event": ev,
                                   "checks": checks.pending}
        return True

    @staticmethod
    def drop_prepared() -> None:
        """Extension: drops prepare_encrypt's preparation (the class's: the node's H(t_k)^key factor and
        its int pool), its factor zeroed in HBM first -- with the ciphertext the node sends, that factor
        decrypts the node's individual update (c / F = 1 + N x).  The encrypt that takes it spends it, a
        call of another round drops it, an encrypt that raises drops it, and so does
        _device.jl_clear_caches (the clear-caches path).  A researcher's prepare_aggregate preparation is
        its instance's (drop it with `crypter.drop_prepared_aggregate()`)."""
        prep, SecaggCrypter._enc_prep = SecaggCrypter._enc_prep, None
        _scrub_prep(prep, ("factor",))

    def drop_prepared_aggregate(self) -> None:
        """Extension: drops this instance's prepare_aggregate preparation, its factors zeroed first."""
        prep, self._prepared = getattr(self, "_prepared", None), None
        _scrub_prep(prep, ("factors",))

    def _take_prepared_encrypt(self, current_round, num_nodes, key, biprime, target_range, n_ct, dev):
        """(prepare_encrypt's factor, its int pool or None) when they are this call's (the factor waited for
        on the current stream, its status words adopted; the preparation is then spent), else None.  A call
        of another round drops it."""
        prep = SecaggCrypter._enc_prep
        if prep is None:
            return None
        if prep["round"] != current_round:
            SecaggCrypter.drop_prepared()
            return None
        tag = _prep_tag(current_round, num_nodes, key, biprime, target_range)
        if prep["n_ct"] != n_ct or tag is None or prep["tag"] != tag:
            return None
        SecaggCrypter._enc_prep = None
        main = torch.cuda.current_stream(dev)
        main.wait_event(prep["event"])
        prep["factor"].record_stream(main)
        D.adopt_checks(prep["checks"])
        return prep["factor"], prep["pool"]

    def prepare_aggregate(self, current_round: int, num_nodes: int, key: int, biprime: int,
                          num_expected_params: int, target_range: Optional[int] = None) -> bool:
        """Extension (not in the reference): issue the decryption factor of a coming `aggregate` now.
        The factor H(t_k)^key of every ciphertext depends only on the round, the server key, the
        biprime and the vector's size, which the researcher knows when it sends the training request
        (`researcher/secagg/_secure_aggregation.py`), so its exponentiations -- most of the aggregate's
        GPU time -- can run on a side stream while the nodes train.  The next `aggregate` of the same
        round, key, biprime, node count, target range and ciphertext count takes it (once); other calls
        of that round leave it, a call of another round drops it.  A device condition of the early work
        is raised by the aggregate that takes it.  It also warms the aggregate's pinned staging buffers
        and makes its output list's float objects (~320 MB of host memory at 10M, held until used or
        dropped), whose values the aggregate then writes in place: with both, the list aggregate at 10M x 8
        takes 45 ms instead of 158 (`profiles/archive/r5x_bench.json`).
        Best effort: False (nothing prepared) where aggregate would refuse the arguments.  The key
        itself is not kept, only a SHA-256 tag of it."""
        self.drop_prepared_aggregate()
        try:
            if not all(isinstance(v, int) for v in (current_round, num_nodes, key, biprime, num_expected_params)):
                return False
            if num_nodes < 1:
                return False
            _, cr = D.jl_slot(target_range or SAParameters.TARGET_RANGE, num_nodes)
            n_ct = -(-num_expected_params // cr)
            if n_ct <= 0:
                return False
            dev = D.device()
            stripes = D.list_encrypt_stripes(n_ct, dev)
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side), D.capture_checks() as checks:
                factors = [self.decrypt_factor_tensor(current_round, c1 - c0, key, biprime, ct_offset=c0)
                           for c0, c1 in stripes]
            ev = torch.cuda.Event()
            ev.record(side)
            # the aggregate's pinned staging buffers, allocated now and handed back to torch's caching host
            # allocator, which gives them to the aggregate: page-locking ~1 GB is the first call's largest
            # extra cost (315-322 ms against 172 ms warm at 10M x 8)
            warm = [D.host_empty((num_nodes, c1 - c0, 64), torch.int32) for c0, c1 in stripes]
            warm += [D.host_empty(((c1 - c0) * cr,), torch.float64) for c0, c1 in stripes]
            del warm
            # and its output list: the float objects made now, their values written in place by the
            # aggregate (making 10M Python floats is most of its host time, ~100 ms)
            pool = D.float_pool(max(0, min(num_expected_params, n_ct * cr)))
        except Exception:  # noqa: BLE001 -- aggregate raises whatever it is, in the reference's order
            return False
        self._prepared = {"round": current_round, "tag": _prep_tag(current_round, num_nodes, key, biprime, target_range),
                          "n_ct": n_ct, "pool": pool,
                          "stripes": stripes, "factors": factors, "event": ev, "checks": checks.pending}
        return True

    def _take_prepared(self, current_round, num_nodes, key, biprime, target_range, n_ct, dev):
        """The prepared factors when they are this call's (waited for on the current stream, their status
        words adopted by the call's deferred checks; the preparation is then spent), else None.  A call of
        the same round that is not the prepared one -- the researcher's insecure-validation aggregate of the
        encryption factors (num_expected_params = 1, `_secure_aggregation.py:372-375`) comes first -- leaves
        it in place; a call of another round drops it."""
        prep = getattr(self, "_prepared", None)
        if prep is None:
            return None
        if prep["round"] != current_round:
            self.drop_prepared_aggregate()
            return None
        tag = _prep_tag(current_round, num_nodes, key, biprime, target_range)
        if prep["n_ct"] != n_ct or tag is None or prep["tag"] != tag:
            return None
        self._prepared = None
        main = torch.cuda.current_stream(dev)
        main.wait_event(prep["event"])
        for f in prep["factors"]:
            f.record_stream(main)
        D.adopt_checks(prep["checks"])
        return prep["stripes"], prep["factors"], prep["pool"]

    def aggregate(self, current_round: int, num_nodes: int, params: List[List[int]], key: int, biprime: int,
                  total_sample_size: int, clipping_range: Union[int, None] = None, num_expected_params: int = 1,
                  target_range: Optional[int] = None) -> List[float]:
        """Decrypts the sum of the parties' ciphertexts (reference `_secagg_crypter.py:139-230`)."""
        start = time.process_time()
        if len(params) != num_nodes:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: Num of parameters that are received from nodes "
                f"does not match the number of nodes has been set for the encrypter. There might "
                f"be some nodes did not answered to training request or num of clients of "
                "`ParameterEncrypter` has not been set properly before train request.")
        with D.deferred_checks():
            # The decryption factor H(t_k)^key needs no ciphertext: issue it first, so the GPU
            # exponentiates while the host validates and converts the parties' lists.  Only
            # when the arguments are well-formed; any error is raised below, in the order
            # the reference raises it.  Vectors of two one-lane rounds or more run as ct_offset
            # stripes (the node encrypt's): stripe k's factor, then its combine and D2H, then
            # stripe k + 1's factor, so the host builds stripe k's floats while the GPU
            # exponentiates stripe k + 1 (every element depends on its own ciphertext only: the
            # stripes' outputs concatenate to the unsplit call's).
            stripes, factors, pool = None, [], None
            if params and isinstance(key, int) and isinstance(biprime, int) and all(isinstance(p, list) for p in params):
                n_ct0 = min(len(p) for p in params)
                if n_ct0:
                    prep = self._take_prepared(current_round, num_nodes, key, biprime, target_range, n_ct0,
                                               D.device())
                    if prep is not None:  # prepare_aggregate's factors (every stripe's) and output list
                        stripes, factors, pool = prep[0], list(prep[1]), prep[2]
                    else:
                        stripes = D.list_encrypt_stripes(n_ct0, D.device())
                        factors = [None] * len(stripes)
                        try:
                            c0, c1 = stripes[0]
                            factors[0] = self.decrypt_factor_tensor(current_round, c1 - c0, key, biprime,
                                                                    ct_offset=c0)
                        except Exception:  # noqa: BLE001 -- re-raised by the regular path below
                            stripes = None

            _check_int_lists(params)
            if not isinstance(key, int):
                raise TypeError("The key should be type of integer")
            if not params:
                raise FedbiomedSecaggCrypterError(
                    f"{ErrorNumbers.FB624.value}: The aggregation of encrypted parameters "
                    f"is not successful: list_y_u_tau should be a non-empty list.")
            n2 = biprime * biprime
            n_ct = min(len(p) for p in params)  # zip(*list_y_u_tau) truncates (_jls.py:691-693)
            if n_ct == 0:
                return []
            dev = D.device()
            if stripes is None:
                stripes, factors = [(0, n_ct)], [None]
            res = self._aggregate_stripes(current_round, params, key, biprime, total_sample_size, clipping_range,
                                          num_expected_params, target_range, n2, n_ct, stripes, factors, dev, pool)
        logger.info(f"Aggregating {len(params)} parameters from {num_nodes} nodes.")
        logger.debug(f"Aggregation is completed in {round(time.process_time() - start, ndigits=2)} seconds.")
        return res

    def _aggregate_stripes(self, current_round, params, key, biprime, total_sample_size, clipping_range,
                           num_expected_params, target_range, n2, n_ct, stripes, factors, dev,
                           pool=None) -> List[float]:
        """The list API's aggregate over ct_offset stripes (one when the vector is small).  Per stripe: the
        parties' ints -> pinned limbs -> H2D on a copy stream, the combine with that stripe's factor, the
        float64 D2H in stream order, then the next stripe's factor.  The host converts every stripe's ints
        first (host threads, one GIL-held C call each: no per-item pins) and issues its GPU work, then makes
        the output list and the last stripe's float objects while the GPU runs the factors (the 10M-element
        float list is the call's largest host cost) and writes each stripe's values as its D2H lands.
        Stripe outputs: elements [c0 cr, c1 cr) capped by
        num_expected_params, as the unsplit decode (_jls.py:146-167); a stripe past it still runs its
        checks (the unsplit call's errors).  `pool`: prepare_aggregate's output list (its floats made
        ahead, written in place here) when it has this call's length."""
        _, cr = D.jl_slot(target_range or SAParameters.TARGET_RANGE, len(params))
        n_exp = int(num_expected_params)
        n_outs = [max(0, min(n_exp - c0 * cr, (c1 - c0) * cr)) for c0, c1 in stripes]
        offs = [sum(n_outs[:k]) for k in range(len(stripes))]
        packed = wire.packed_rows(params, "jl", n_ct)

        def stage(k):  # stripe k's limbs in a pinned buffer: its H2D is then truly asynchronous
            c0, c1 = stripes[k]
            staged = D.host_empty((len(params), c1 - c0, 64), torch.int32)
            limbs = staged.numpy().view(np.uint32)
            if packed is not None:
                limbs[:] = packed[:, c0:c1]
            return staged, limbs

        keep = []
        main = torch.cuda.current_stream(dev)
        copy = torch.cuda.Stream(device=dev)
        S = len(stripes)

        def issue(k):  # stripe k's H2D -> combine -> D2H, then stripe k + 1's factor behind the combine
            c0, c1 = stripes[k]
            staged = bufs[k][0]
            with torch.cuda.stream(copy):
                cts = staged.to(dev, non_blocking=True)
            main.wait_stream(copy)
            cts.record_stream(main)
            keep.append(staged)
            if factors[k] is None and S > 1:
                factors[k] = self.decrypt_factor_tensor(current_round, c1 - c0, key, biprime, ct_offset=c0)
            out = self.aggregate_tensor(current_round, cts, key, biprime, total_sample_size, clipping_range,
                                        n_outs[k], target_range, ct_offset=c0, decrypt_factor=factors[k])
            out_h = D.host_empty(out.shape, torch.float64)
            out_h.copy_(out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(main)
            if k + 1 < S and factors[k + 1] is None:
                n0, n1 = stripes[k + 1]
                factors[k + 1] = self.decrypt_factor_tensor(current_round, n1 - n0, key, biprime, ct_offset=n0)
            return out_h, ev

        # Every stripe's ints are converted (host threads, one GIL-held C call each) and its H2D -> combine
        # -> D2H issued first; then, while the GPU runs the factors, the output list and the last stripe's
        # float objects are made (prepared: all of them were made ahead); each stripe's floats are made with
        # their values as its D2H lands, the last stripe's values written in place -- so the host's largest
        # cost, the 10M float objects, runs beside the factors instead of after the last one.
        bufs, pend = [None] * S, []
        for k in range(S):
            bufs[k] = stage(k)
            if packed is None:
                D.convert_stripe(params, *stripes[k], n2, bufs[k][1])
            pend.append(issue(k))
        if pool is not None and len(pool) == sum(n_outs):
            res = pool
        else:  # the last stripe's float objects made now (its values land last); the others' as they land
            res = D.none_list(sum(n_outs))
            if D.inplace(prepared=False, call="aggregate"):
                D.f64_into_list(res, offs[-1], np.zeros(n_outs[-1]))
        for k, (out_h, ev) in enumerate(pend):
            ev.synchronize()
            D.f64_into_list(res, offs[k], out_h.numpy())
        return res

    @staticmethod
    def _apply_average(params: List[int], total_weight: int) -> List:
        """Reference `_secagg_crypter.py:233-249` on the device (`fbm_int_ops`: integer sums below
        2^128; an integer divisor of either sign below 2^64 in magnitude, or a float one, never
        truncated); the crypters' own averaging is fused into their kernels."""
        if any(v < 0 for v in params):
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: Cannot compute weighted average, values outside of bounds")
        if not params:
            return []
        return D.int_true_divide(D.ints_to_u128(params), total_weight)  # its ZeroDivisionErrors as Python's

    @staticmethod
    def _apply_weighting(params: List[int], weight: int, target_range: int = SAParameters.TARGET_RANGE) -> List[int]:
        """Reference `_secagg_crypter.py:252-276` on the device (`fbm_int_ops`: values below 2^128, a
        weight of either sign below 2^64 in magnitude, exact products); the crypters' own weighting
        is fused into their encrypt kernels."""
        max_val = target_range - 1
        if any(v > max_val or v < 0 for v in params):
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: Cannot apply weight to parameters, values outside of bounds")
        if not params:
            return []
        return D.int_multiply(D.ints_to_u128(params), weight)


class SecaggLomCrypter(SecaggCrypter):
    """Low-Overhead Masking secure aggregation (reference `_secagg_crypter.py:300-455`)."""

    def prepare_aggregate(self, *args, num_params: Optional[int] = None, **kwargs) -> bool:
        """Extension (not in the reference): `prepare_aggregate(num_params)`.  LOM's aggregate is a sum with
        no exponentiation, so nothing runs ahead on the device; what is made ahead is the output list's
        float objects (`float_pool`), whose values the next `aggregate` of `num_params` values writes in
        place (making 10M Python floats is ~100 ms of the call).  An aggregate of another size -- the
        researcher's one-value validation aggregate comes first (`_secure_aggregation.py:372-387`) --
        leaves it.  False (nothing prepared) for anything but one positive int: the Joye-Libert form
        (round, nodes, key, biprime, size) has no LOM counterpart."""
        self._lom_agg_pool = None
        if num_params is None and len(args) == 1:
            num_params = args[0]
        elif args:
            return False
        if not isinstance(num_params, int) or isinstance(num_params, bool) or num_params <= 0:
            return False
        self._lom_agg_pool = D.float_pool(num_params)
        return True

    def prepare_encrypt(self, current_round: int, node_id: str, num_params: int) -> bool:
        """Extension (not in the reference): make the next `encrypt`'s output list ahead -- its int objects
        (`int_pool`), whose values the encrypt of that round, node and size writes in place (making 10M
        Python ints is most of a 10M-element list encrypt).  Nothing secret is computed or kept.  False
        (nothing prepared) where the pool cannot be made (CPython >= 3.12 builds) or for bad arguments."""
        self._lom_enc_prep = None
        if not isinstance(num_params, int) or isinstance(num_params, bool) or num_params <= 0:
            return False
        pool = D.int_pool(num_params, 8)
        if pool is None:
            return False
        self._lom_enc_prep = {"round": current_round, "node_id": node_id, "n": num_params, "pool": pool}
        return True

    def _take_enc_pool(self, current_round, node_id, n):
        prep = getattr(self, "_lom_enc_prep", None)
        if prep is None or prep["round"] != current_round or prep["node_id"] != node_id or prep["n"] != n:
            return None
        self._lom_enc_prep = None
        return prep["pool"]

    def __init__(self, nonce: Optional[str] = None):
        if nonce:
            nonce = str.encode(nonce).zfill(16)[:16]
        self._nonce: bytes = nonce if nonce else secrets.token_bytes(16)

    @property
    def nonce(self) -> bytes:
        return self._nonce

    def encrypt_tensor(self, current_round: int, node_id: str, params: torch.Tensor,
                       pairwise_secrets: Dict[str, bytes], node_ids: List[str],
                       clipping_range: Union[int, None] = None, weight: Optional[int] = None,
                       target_range: Optional[int] = None, elem_offset: int = 0,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Device tensor (f32/f64) -> masked uint64 vector (int64 tensor) in HBM.
        `elem_offset`: global index of this shard's first element (multiple of 8); `out`: an
        int64 destination (e.g. this party's row of the [P, n] matrix aggregate_tensor takes)."""
        target_range = target_range or SAParameters.TARGET_RANGE
        _check_weight(weight, jl=False)
        if params.numel() == 0:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value} Error during parameter encryption. max() arg is an empty sequence")
        secrets_, signs = self._peer_masks(node_id, pairwise_secrets, node_ids)
        if weight is None or weight >= 0:
            return D.lom_protect(params, secrets_, signs, self._nonce, current_round, len(node_ids),
                                 clip=clipping_range, target=target_range, weight=1 if weight is None else weight,
                                 elem_offset=elem_offset, out=out)
        # Negative weight: LOM.protect's overflow guard sees bit_length(q*w) == bit_length(q*|w|)
        # (_lom.py:133-150), then np.array(x_u_tau, dtype=uint64) raises OverflowError at the
        # first negative product (_lom.py:153; not wrapped by the crypter, which only catches
        # TypeError / ValueError).  All-zero products pass and mask nothing but zeros.
        y = D.lom_protect(params, secrets_, signs, self._nonce, current_round, len(node_ids),
                          clip=clipping_range, target=target_range, weight=-weight, elem_offset=elem_offset,
                          out=out, check_now=True)
        q = D.lom_protect(params, [], [], bytes(16), 0, 0, clip=clipping_range, target=target_range, weight=1,
                          check_now=True)
        nz = torch.nonzero(q)
        if nz.numel():
            qv = int(q[int(nz[0, 0])].item()) & D.U64_MAX
            raise OverflowError(f"Python integer {qv * weight} out of bounds for uint64")
        return y

    @staticmethod
    def _peer_masks(node_id: str, pairwise_secrets: Dict[str, bytes], node_ids: List[str]):
        """The peers' pairwise secrets in node order and their mask signs (LOM.protect, _lom.py:151-173)."""
        peers = [p for p in node_ids if p != node_id]
        secrets_ = [pairwise_secrets[p] for p in peers]
        signs = [1 if p < node_id else -1 for p in peers]
        if len(node_ids) == 0:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value} Error during parameter encryption. math domain error")
        return secrets_, signs

    def aggregate_tensor(self, Y: torch.Tensor, total_sample_size: int, clipping_range: Union[int, None] = None,
                         target_range: Optional[int] = None, want_sums: bool = False):
        """[P, n] masked vectors in HBM -> float64 [n] averaged parameters."""
        out, sums = D.lom_aggregate(Y, total_sample_size, clipping_range, target_range or SAParameters.TARGET_RANGE,
                                    want_sums=want_sums)
        return (out, sums) if want_sums else out

    def encrypt(self, current_round: int, node_id: str, params: List[float], pairwise_secrets: Dict[str, bytes],
                node_ids: List[str], clipping_range: Union[int, None] = None, weight: Optional[int] = None,
                target_range: Optional[int] = None) -> List[int]:
        start = time.process_time()
        host = _check_float_list(params)
        target_range = target_range or SAParameters.TARGET_RANGE
        if params:  # quantize() evaluates nothing on an empty list
            D.quant_params(clipping_range, target_range)
        _check_weight(weight, jl=False)  # before LOM.protect's empty-input error, as the reference
        if not params:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value} Error during parameter encryption. max() arg is an empty sequence")
        if len(params) <= D.LOM_HOST_CALL_MAX and (weight is None or weight >= 0):
            # a small vector: copy in, kernel, copy out and status in one synchronous C call
            secrets_, signs = self._peer_masks(node_id, pairwise_secrets, node_ids)
            packed = D.lom_protect_host(host.numpy(), secrets_, signs, self._nonce, current_round, len(node_ids),
                                        clip=clipping_range, target=target_range,
                                        weight=1 if weight is None else weight)
        else:
            with D.deferred_checks():  # the status word checked once the masked vector is back (one sync per call)
                x = host.to(D.device(), non_blocking=True)
                y = self.encrypt_tensor(current_round, node_id, x, pairwise_secrets, node_ids, clipping_range,
                                        weight, target_range)
                packed = D.to_host(y).numpy().view(np.uint64)
        pool = self._take_enc_pool(current_round, node_id, packed.shape[0])
        out = D.u64_into_pool(pool, packed) if pool is not None else packed.tolist()
        if wire.enabled():
            out = wire.EncryptedParams(out, "lom", packed)
        logger.debug(f"Encryption of the parameters took {time.process_time() - start} seconds.")
        return out

    def aggregate(self, params: List[List[int]], total_sample_size: int, clipping_range: Union[int, None] = None,
                  target_range: Optional[int] = None) -> List[float]:
        start = time.process_time()
        _check_int_lists(params)
        num_nodes = len(params)
        packed = wire.packed_rows(params, "lom")
        dev = D.device()
        try:
            Yh, pinned = (torch.from_numpy(packed.view(np.int64)), False) if packed is not None else \
                D.u64_to_host(params)
        except (ValueError, TypeError) as e:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: The aggregation of encrypted parameters "
                f"is not successful: {e}") from e
        if Yh.dim() != 2 or Yh.shape[1] == 0:
            return []
        if Yh.shape[1] <= D.LOM_HOST_CALL_MAX:  # a small vector: one synchronous C call, host to host
            res_h = D.lom_aggregate_host(Yh.numpy().view(np.uint64), total_sample_size, clipping_range,
                                         target_range or SAParameters.TARGET_RANGE)
        else:
            with D.deferred_checks():  # the status word checked once the averages are back
                out = self.aggregate_tensor(Yh.to(dev, non_blocking=pinned), total_sample_size, clipping_range,
                                            target_range)
                res_h = D.to_host(out).numpy()
        logger.info(f"Aggregating {len(params)} parameters from {num_nodes} nodes.")
        pool = getattr(self, "_lom_agg_pool", None)
        if pool is not None and len(pool) == res_h.shape[0]:  # prepare_aggregate's floats, written in place
            self._lom_agg_pool = None
            D.f64_into_list(pool, 0, res_h)
            res = pool
        else:
            res = res_h.tolist()
        logger.debug(f"Aggregation is completed in {round(time.process_time() - start, ndigits=2)} seconds.")
        return res


D._clear_hooks.append(SecaggCrypter.drop_prepared)  # _device.jl_clear_caches drops the node's prepared factor
