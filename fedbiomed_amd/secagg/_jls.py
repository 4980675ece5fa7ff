"""Joye-Libert objects mirroring the reference class API (fedbiomed/common/secagg/_jls.py):
VES, PublicParam, EncryptedNumber, BaseKey, UserKey, ServerKey, JoyeLibert and FDH, for
callers and tests that use them directly (SecaggCrypter itself runs the fused tensor path).

Every vector operation runs in the gfx950 kernels through the C-ABI (include/fbm_secagg.h):

    VES.encode / VES.decode           fbm_jl_pack / fbm_jl_unpack        _jls.py:118-192
    FDH.H, BaseKey._populate_tau      fbm_jl_fdh                         _jls.py:451-467, 727-762
    UserKey.encrypt                   fbm_jl_encrypt (FBM_PT)            _jls.py:473-505
    EncryptedNumber sums              fbm_jl_product                     _jls.py:308-374
    ServerKey.decrypt                 fbm_jl_decrypt                     _jls.py:520-562
    JoyeLibert.protect                fbm_jl_encrypt (FBM_U128)          _jls.py:593-644
    JoyeLibert.aggregate              fbm_jl_aggregate (decoded sums)    _jls.py:646-699

A sum of EncryptedNumbers keeps its operands until its ciphertext is read (then one device
product), so `[sum(ep) for ep in zip(*parties)]` followed by ServerKey.decrypt is one device
call, as JoyeLibert.aggregate is.

A PublicParam whose hashing function is anything but FDH(2048, N^2).H with bits = 1024 (what
SecaggCrypter._setup_public_param builds) has its hashes computed as the reference computes them --
the callable per t on the host (one fbm_jl_fdh launch for an FDH of bits_size 2048 against another
modulus) -- and the exponentiations on the device (fbm_jl_powmod / fbm_jl_decrypt_with).

Domain of the device path (FB624 outside it): 1 <= N < 2^1024 (an even N and
N = 1 run on the generic engine, fedbiomed_amd/csrc/fbm_gen.hip, an odd one on the Montgomery engines);
FDH of any bits_size (an r of up to 255 digests, round 5); tau in [0, 2^8192) where FDH hashes it; VES
values of any width and sign, any slot and plaintext size (rounds 4-5); ServerKey.decrypt with any invertible
delta (round 5).  Integers are Python ints (gmpy2 is
not a dependency): where the reference returns gmpy2.mpz this returns int, and FDH takes an
int modulus.
"""

import math
import operator
from typing import Callable, List, Optional, Tuple, Union

import numpy as np
import torch

from .. import _device as D
from ..constants import ErrorNumbers, SAParameters
from ..exceptions import FedbiomedSecaggCrypterError

_TAU_SHIFT_BITS = SAParameters.KEY_SIZE // 2  # PublicParam.bits of SecaggCrypter._setup_public_param


def _unsupported(what: str) -> FedbiomedSecaggCrypterError:
    return FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: {what} is outside the device path's domain")


def _is_integer(v) -> bool:
    return (isinstance(v, int) and not isinstance(v, bool)) or type(v).__name__ == "mpz"


class VES:
    """The vector encoding class (reference _jls.py:76-192): packs `comp_ratio` values of
    `element_size` bits into one plaintext, on the device."""

    def __init__(self, ptsize: int, valuesize: int) -> None:
        self._ptsize: int = ptsize
        self._valuesize: int = valuesize

    def _get_elements_size_and_compression_ratio(self, add_ops: int) -> Tuple[int, int]:
        """reference _jls.py:104-116"""
        element_size = self._valuesize + math.ceil(math.log2(add_ops + 1))
        comp_ratio = math.floor(self._ptsize / element_size)
        return element_size, comp_ratio

    def _slot(self, add_ops: int) -> Tuple[int, int]:
        """(element_size, comp_ratio); comp_ratio 0 when a slot is wider than the plaintext (encode then packs
        every value into one plaintext -- the reference's bs never reaches 0 -- and decode reads none)."""
        return self._get_elements_size_and_compression_ratio(add_ops)

    def encode(self, V: List[int], add_ops: int) -> List[int]:
        """reference _jls.py:118-144 (OR packing, _batch :169-176) -- fbm_jl_pack for the crypter's shape
        (es <= 100, es * cr <= 1024, values < 2^128), fbm_ves_pack for any other (round 4)."""
        es, cr = self._slot(add_ops)
        if not V:
            return []
        V = [operator.index(v) for v in V]
        if cr < 1:  # bs = 0 - 1 - 1 ... never reaches 0: one plaintext holds every value (round 5)
            return D.ves_pack_any(V, es, len(V))
        wmax = max(v.bit_length() for v in V)
        if es <= 100 and es * cr <= 1024 and wmax <= 128 and es * (cr - 1) + wmax <= 1024 and min(V) >= 0:
            pt = D.jl_pack(D.ints_to_u128(V), es, cr)  # (no bit of any plaintext past 2^1024)
            return D.limbs_to_ints_w(pt, 32)
        return D.ves_pack_any(V, es, cr)  # any width, negative values included (round 5)

    def decode(self, E: List[int], add_ops: int, v_expected: int) -> List[int]:
        """reference _jls.py:146-167 (_debatch :179-192): slot j = (e >> es*j) & (2^es - 1),
        min(remaining, comp_ratio) values per plaintext -- fbm_jl_unpack for the crypter's shape,
        fbm_ves_unpack for any other (round 4)."""
        es, cr = self._slot(add_ops)
        if not E or v_expected <= 0 or cr < 1:  # comp_ratio 0: min(v_expected, 0) values per plaintext
            return []
        if es > 128 or es * cr > 1024:
            return D.ves_unpack_any([int(e) for e in E], es, cr, v_expected)
        # only the low es*cr <= 1024 bits of a plaintext are read: two's-complement truncation
        pts = D.ints_to_pt([int(e) & ((1 << 1024) - 1) for e in E], 1 << 1024)
        return D.u128_to_ints(D.jl_unpack(pts, es, cr, v_expected))


class PublicParam:
    """The public parameters for Joye-Libert Scheme (reference _jls.py:195-286)."""

    def __init__(self, n_modulus: int, bits: int, hashing_function: Callable) -> None:
        self._n_modulus = n_modulus
        self._n_square = n_modulus * n_modulus
        self._bits = bits
        self._hashing_function = hashing_function

    @property
    def bits(self) -> int:
        return self._bits

    @property
    def n_modulus(self) -> int:
        return self._n_modulus

    @property
    def n_square(self) -> int:
        return self._n_square

    def hashing_function(self, val: int):
        return self._hashing_function(val)

    def __eq__(self, other: "PublicParam") -> bool:
        return self._n_modulus == other.n_modulus

    __hash__ = None  # as the reference: __eq__ without __hash__

    def __repr__(self) -> str:
        hashcode = hex(hash(self._hashing_function))
        n_str = str(int(self._n_modulus))
        return "<PublicParam (N={}...{}, H(x)={})>".format(n_str[:5], n_str[-5:], hashcode[:10])


def _fdh_standard(pp: PublicParam) -> bool:
    """Is pp's hashing function FDH(2048, N^2).H with bits 1024 (SecaggCrypter._setup_public_param's)?
    Then the fused entry points hash on the device inside the encrypt / decrypt call."""
    fdh = getattr(pp._hashing_function, "__self__", None)
    return (isinstance(fdh, FDH) and getattr(pp._hashing_function, "__func__", None) is FDH.H
            and fdh.bits_size == SAParameters.KEY_SIZE and _is_integer(fdh._n_modules)
            and int(fdh._n_modules) == int(pp.n_modulus) ** 2 and pp.bits == _TAU_SHIFT_BITS)


def _bases(key: "BaseKey", tau, len_: int, n: int) -> torch.Tensor:
    """Any other hashing function: BaseKey._populate_tau's values (the callable per t on the host, as
    the reference calls it, or one fbm_jl_fdh launch for an FDH of another modulus) as device limbs of
    the powmod bases; a base outside [0, 2^2048) is reduced mod N^2 (gmpy2.powmod reduces its base)."""
    vals = [operator.index(h) for h in key._populate_tau(tau, len_)]  # a non-integer: TypeError
    return torch.from_numpy(D.ints_to_limbs(vals, n * n).view(np.int32)).to(D.device())


def _check_tau(tau) -> int:
    """A round: any 0 <= tau < 2^8192 (the device hashes t = (k << 512) | tau whole, ABI 3).  A negative
    one, or one of 2^8192 or more, is the reference's OverflowError (FDH.H's int(t).to_bytes(1024),
    _jls.py:747)."""
    t = operator.index(tau)
    if t < 0:
        raise OverflowError("can't convert negative int to unsigned")
    if t >> D.JL_ROUND_BITS:
        raise OverflowError("int too big to convert")
    return t


class EncryptedNumber(object):
    """An encrypted number by one of the user keys (reference _jls.py:289-374).  A sum keeps
    its operands until `ciphertext` is read: the product mod N^2 then runs on the device."""

    def __init__(self, param: PublicParam, ciphertext: int):
        self.public_param = param
        self.ciphertext = ciphertext

    @classmethod
    def _of_terms(cls, param: PublicParam, terms: Tuple[int, ...]) -> "EncryptedNumber":
        e = cls.__new__(cls)
        e.public_param = param
        e._terms, e._value = terms, None
        return e

    @property
    def ciphertext(self) -> int:
        if self._value is None:
            self._value = _materialize([self])[0]
            self._terms = (self._value,)
        return self._value

    @ciphertext.setter
    def ciphertext(self, value) -> None:
        v = int(value)  # gmpy2.mpz(value) in the reference
        self._terms, self._value = (v,), v

    def __add__(self, other: "EncryptedNumber") -> "EncryptedNumber":
        if not isinstance(other, EncryptedNumber):
            raise TypeError(
                "Encrypted number can be only summed with another Encrypted num."
                f"Can not sum Encrypted number with type {type(other)}"
            )
        return self._add_encrypted(other)

    def __iadd__(self, other):
        return self.__add__(other)

    def __radd__(self, other: Union["EncryptedNumber", int]) -> "EncryptedNumber":
        if other == 0:
            return self
        return self.__add__(other)

    def __repr__(self) -> str:
        r = str(self.ciphertext)
        return "<EncryptedNumber {}...{}>".format(r[:5], r[-5:])

    def _add_encrypted(self, other: "EncryptedNumber") -> "EncryptedNumber":
        if self.public_param != other.public_param:
            raise ValueError("Attempted to add numbers encrypted against different parameters!")
        return EncryptedNumber._of_terms(self.public_param, self._terms + other._terms)


def _term_rows(nums: List[EncryptedNumber], n: int) -> torch.Tensor:
    """int32 [P, len(nums), 64] limbs of the numbers' product operands, shorter products
    padded with the identity 1 (P = the most operands of any number)."""
    P = max((len(e._terms) for e in nums), default=1)
    host = D.host_empty((P, len(nums), 64), torch.int32)
    buf = host.numpy().view(np.uint32)
    for u in range(P):
        col = [e._terms[u] if u < len(e._terms) else 1 for e in nums]
        D.ints_to_limbs(col, n * n, out=buf[u])
    return host.to(D.device())


def _sum_column(col) -> Union[EncryptedNumber, int]:
    """sum(col) with the reference's operand and parameter checks (_jls.py:308-374, 691-693);
    no arithmetic: the sum carries every operand to the device product."""
    if col and all(type(e) is EncryptedNumber for e in col):
        p0 = col[0].public_param
        if all(e.public_param is p0 for e in col) or all(p0 == e.public_param for e in col[1:]):
            if len(col) == 1:
                return col[0]
            return EncryptedNumber._of_terms(p0, tuple(t for e in col for t in e._terms))
    acc = 0
    for e in col:  # the general case, raising where sum() raises
        acc = acc + e
    return acc


def _materialize(nums: List[EncryptedNumber]) -> List[int]:
    """Ciphertexts of (lazy) sums: one device product over all of them."""
    n = _modulus_of(nums[0].public_param)
    return D.limbs_to_ints(D.to_host(D.jl_product(_term_rows(nums, n), n)).numpy())


def _modulus_of(pp: PublicParam) -> int:
    n = int(pp.n_modulus)
    if n < 1 or n.bit_length() > 1024:
        raise _unsupported("a modulus N outside [1, 2^1024)")
    return n


class BaseKey:
    """A base key class for Joye-Libert Scheme (reference _jls.py:377-467)."""

    def __init__(self, public_param: PublicParam, key: int):
        if not isinstance(key, int):
            raise TypeError("The key should be type of integer")
        self._public_param = public_param
        self._key = int(key)

    @property
    def public_param(self) -> PublicParam:
        return self._public_param

    @property
    def key(self) -> int:
        return self._key

    def __repr__(self):
        hashcode = hex(hash(self))
        return "<ServerKey {}>".format(hashcode[:10])

    def __eq__(self, other: Union["BaseKey", "ServerKey", "UserKey"]) -> bool:
        if not isinstance(other, type(self)):
            raise TypeError(f"The key can not be compared with type {type(other)}")
        return self._public_param == other.public_param and self._key == other.key

    def __hash__(self) -> int:
        return hash(self._key)

    def _populate_tau(self, tau: int, len_: int):
        """reference _jls.py:451-467: [H((k << bits/2) | tau) for k < len_] -- one fbm_jl_fdh
        launch when the hashing function is an FDH of bits_size 2048 and bits is 1024; any
        other hashing function is the caller's own callable and is called per t."""
        pp = self._public_param
        fdh = getattr(pp._hashing_function, "__self__", None)
        if (isinstance(fdh, FDH) and getattr(pp._hashing_function, "__func__", None) is FDH.H
                and pp.bits == _TAU_SHIFT_BITS):
            return fdh._hash_range(tau, len_)
        return [pp.hashing_function((k << (pp.bits // 2)) | tau) for k in range(len_)]


class UserKey(BaseKey):
    """A user key for Joye-Libert Scheme (reference _jls.py:470-505)."""

    def encrypt(self, plaintext: List[int], tau: int) -> List[int]:
        """c_k = (N pt_k + 1) H(t_k)^key mod N^2 -- fbm_jl_encrypt on plaintext limbs."""
        if not isinstance(plaintext, list):
            raise TypeError(f"Expected plaintext type list but got {type(plaintext)}")
        if not plaintext:  # the reference hashes no round for an empty list
            return []
        n = _modulus_of(self._public_param)
        if not _fdh_standard(self._public_param):  # the caller's hashing function, then fbm_jl_powmod
            pts = D.ints_to_pt(plaintext, n)
            ct = D.jl_powmod(_bases(self, tau, len(plaintext), n), n, self._key, pts)
            return D.limbs_to_ints(D.to_host(ct).numpy())
        tau = _check_tau(tau)
        pts = D.ints_to_pt(plaintext, n)
        ct = D.jl_encrypt(pts, n, self._key, tau, 1, kind="pt")
        return D.limbs_to_ints(D.to_host(ct).numpy())


class ServerKey(BaseKey):
    """A server key for Joye-Libert Scheme (reference _jls.py:508-562)."""

    def __init__(self, public_param: PublicParam, key: int) -> None:
        super().__init__(public_param, key)

    def decrypt(self, cipher: List[EncryptedNumber], tau: int, delta: int = 1) -> List[int]:
        """x_k = ((c_k H(t_k)^(delta^2 key) mod N^2) - 1) // N mod N, times delta^-2 mod N --
        fbm_jl_decrypt (the product of a lazy sum's operands runs in the same call)."""
        if not isinstance(cipher, list):
            raise TypeError(f"Expected `cipher` is list of encrypter numbers but got {type(cipher)}")
        if not all([isinstance(c, EncryptedNumber) for c in cipher]):
            raise TypeError("Cipher text should be list of EncryptedNumbers")
        n = _modulus_of(self._public_param)
        d2 = delta ** 2
        if n == 1 or math.gcd(d2 % (n * n), n * n) != 1:  # invert(delta^2, N^2) runs even on an empty
            raise ZeroDivisionError("invert() no inverse exists")  # list; modulo 1 its result is 0: raises
        if not cipher:
            return []
        if not _fdh_standard(self._public_param):  # fbm_jl_powmod's factor, then fbm_jl_decrypt_with
            rows = _term_rows(cipher, n)
            factor = D.jl_powmod(_bases(self, tau, len(cipher), n), n, d2 * self._key)
            x = D.jl_decrypt_with(rows, n, factor)
        else:
            tau = _check_tau(tau)
            x = D.jl_decrypt(_term_rows(cipher, n), n, d2 * self._key, tau)
        if d2 % n != 1:  # x * invert(delta^2, N^2) mod N (round 5), on the device: see _times_mod_n
            x = _times_mod_n(x, pow(d2, -1, n * n) % n, n)
        return D.limbs_to_ints_w(x, 32)


def _times_mod_n(x: torch.Tensor, c: int, n: int) -> torch.Tensor:
    """c x mod N for plaintext limbs x (int32 [k, 32], x < N) and a constant c, on the device through the
    binomial identity (1 + N x)^c = 1 + N (c x mod N) (mod N^2): fbm_jl_powmod builds 1 + N x (base 1, key 1,
    plaintext x), raises it to c, and fbm_jl_decrypt_with's L(v) = ((v - 1) // N) mod N reads c x mod N back."""
    ones = torch.zeros((x.shape[0], 64), dtype=torch.int32, device=x.device)
    ones[:, 0] = 1
    v = D.jl_powmod(D.jl_powmod(ones, n, 1, x), n, c)
    return D.jl_decrypt_with(v[None], n, ones)


class JoyeLibert:
    """The Joye-Libert scheme (reference _jls.py:565-699): Protect and Agg."""

    def __init__(self, target_range: Optional[int] = None):
        target_range = target_range or SAParameters.TARGET_RANGE
        self._vector_encoder = VES(
            ptsize=SAParameters.KEY_SIZE // 2,
            valuesize=math.ceil(math.log2(target_range) + math.log2(SAParameters.WEIGHT_RANGE)),
        )

    def protect(self, public_param: PublicParam, user_key: UserKey, tau: int, x_u_tau: List[int],
                n_users: int) -> List[int]:
        """y = (1 + x N) H(tau)^sk_u mod N^2 of the VES-packed input -- one fbm_jl_encrypt."""
        if not isinstance(user_key, UserKey):
            raise TypeError(f"Expected key for encryption type is UserKey. but got {type(user_key)}")
        if user_key.public_param != public_param:
            raise ValueError(
                "Bad public parameter. The public parameter of user key does not match the "
                "one given for encryption"
            )
        if not isinstance(x_u_tau, list):
            raise TypeError(
                f"Bad vector for encryption. Excepted argument `x_u_tau` type list but "
                f"got {type(x_u_tau)}"
            )
        es, cr = self._vector_encoder._slot(n_users)
        if not x_u_tau:
            return []
        n = _modulus_of(user_key.public_param)
        wmax = max(operator.index(v).bit_length() for v in x_u_tau)
        if es > 100 or es * cr > 1024 or wmax > 128 or es * (cr - 1) + wmax > 1024 or min(x_u_tau) < 0:
            # a VES shape outside the fused kernels' (a target range past 2^83, values of 2^128 and more):
            # the reference's two steps, VES.encode then UserKey.encrypt, each on the device
            return user_key.encrypt(self._vector_encoder.encode(x_u_tau, n_users), tau)
        if not _fdh_standard(user_key.public_param):  # VES on the device, the caller's hashes, fbm_jl_powmod
            pt = D.jl_pack(D.ints_to_u128(x_u_tau), es, cr)
            ct = D.jl_powmod(_bases(user_key, tau, pt.shape[0], n), n, user_key.key, pt)
            return D.limbs_to_ints(D.to_host(ct).numpy())
        tau = _check_tau(tau)
        ct = D.jl_encrypt(D.ints_to_u128(x_u_tau), n, user_key.key, tau, n_users, slot=(es, cr), kind="u128")
        return D.limbs_to_ints(D.to_host(ct).numpy())

    def aggregate(self, sk_0: ServerKey, tau: int, list_y_u_tau: List[List[EncryptedNumber]],
                  num_expected_params: int) -> List[int]:
        """X = ((prod_u y_u * H(tau)^sk_0 mod N^2) - 1) // N mod N, VES-decoded -- one
        fbm_jl_aggregate (product, server-key factor, decryption and decode on the device)."""
        if not isinstance(sk_0, ServerKey):
            raise ValueError("Key must be an instance of `ServerKey`")
        if not isinstance(list_y_u_tau, list) or not list_y_u_tau:
            raise ValueError("list_y_u_tau should be a non-empty list.")
        if not isinstance(list_y_u_tau[0], list):
            raise ValueError("list_y_u_tau should be a list that contains list of encrypted numbers")
        n_user = len(list_y_u_tau)
        summed = [_sum_column(col) for col in zip(*list_y_u_tau)]  # strict=False: shortest length
        # ServerKey.decrypt's checks, then the decode's slot
        if not all([isinstance(c, EncryptedNumber) for c in summed]):
            raise TypeError("Cipher text should be list of EncryptedNumbers")
        if not summed:
            return []
        n = _modulus_of(sk_0.public_param)
        standard = _fdh_standard(sk_0.public_param)
        if standard:
            tau = _check_tau(tau)
        es, cr = self._vector_encoder._slot(n_user)
        if es > 100 or es * cr > 1024:  # past the fused kernels' slot (fbm_capi build_jl_params): ServerKey.decrypt, VES.decode
            return self._vector_encoder.decode(sk_0.decrypt(summed, tau), n_user, num_expected_params)
        rows = _term_rows(summed, n)
        factor = None if standard else D.jl_powmod(_bases(sk_0, tau, len(summed), n), n, sk_0.key)
        _, sums = D.jl_aggregate(rows, n, sk_0.key, tau, num_expected_params, 1, want_out=False, want_sums=True,
                                 slot=(es, cr), factor=factor)
        return D.u128_to_ints(sums)


class FDH:
    """The Full-Domain Hash scheme (reference _jls.py:702-762), on the device."""

    def __init__(self, bits_size: int, n_modulus: int) -> None:
        if not isinstance(bits_size, int):
            raise TypeError(f"Bits size should be an integer not {type(bits_size)}")
        if not _is_integer(n_modulus):
            raise TypeError(f"n_modules should be of type `gmpy2.mpz` not {type(n_modulus)}")
        self.bits_size = bits_size
        self._n_modules = n_modulus

    def _hash_range(self, tau: int, len_: int, k0: int = 0) -> List[int]:
        if len_ <= 0:
            return []
        if self.bits_size != SAParameters.KEY_SIZE:  # every t_k = (k << 512) | tau in one fbm_jl_fdh_msg launch
            ts = [((k0 + k) << (_TAU_SHIFT_BITS // 2)) | operator.index(tau) for k in range(len_)]
            h = D.jl_fdh_msg(ts, self.bits_size, int(self._n_modules))
            return D.limbs_to_ints_w(h, h.shape[1])
        tau = _check_tau(tau)
        h = D.jl_fdh(len_, int(self._n_modules), tau, k0)
        return D.limbs_to_ints(D.to_host(h).numpy())

    def H(self, t: int) -> int:
        """SHA256(t || 1) || SHA256(t || 2) || ... until gcd(r, n_modulus) == 1, t as bits_size // 2
        big-endian bytes -- fbm_jl_fdh with tau = t and k = 0 at bits_size 2048 (any 0 <= t < 2^8192),
        fbm_jl_fdh_msg at any other bits_size (round 4)."""
        if self.bits_size != SAParameters.KEY_SIZE:
            h = D.jl_fdh_msg([operator.index(t)], self.bits_size, int(self._n_modules))
            return D.limbs_to_ints_w(h, h.shape[1])[0]  # (rows of r's width: up to 255 digests)
        t = _check_tau(t)  # int(t).to_bytes(1024, ...)'s OverflowError outside [0, 2^8192) (_jls.py:747)
        return self._hash_range(t, 1, 0)[0]
