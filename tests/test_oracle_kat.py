"""The CPU restatement's primitives against published known-answer tests (FIPS 180-4 / RFC 1321 / FIPS 197 /
RFC 6229 / RFC 6070) and against Python's hashlib; and str_to_uchar's BN_hex2bn/BN_bn2bin semantics."""
import hashlib
import os
import random

import pytest


def test_sha_family_fips_vectors(oracle):
    assert oracle.sha1(b"abc").hex() == "a9993e364706816aba3e25717850c26c9cd0d89d"
    assert oracle.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert oracle.sha384(b"abc").hex() == ("cb00753f45a35e8bb5a03d699ac65007272c32ab0eded1631a8b605a43ff5bed"
                                           "8086072ba1e7cc2358baeca134c825a7")
    assert oracle.sha512(b"abc").hex() == ("ddaf35a193617abacc417349ae20413112e6fa4e89a97ea20a9eeee64b55d39a"
                                           "2192992a274fc1a836ba3c23a3feebbd454d4423643ce80e2a9ac94fa54ca49f")
    assert oracle.md5(b"abc").hex() == "900150983cd24fb0d6963f7d28e17f72"
    assert oracle.md5(b"").hex() == "d41d8cd98f00b204e9800998ecf8427e"


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 111, 112, 127, 128, 200, 1024, 4480])
def test_sha_md5_vs_hashlib(oracle, n):
    m = bytes(random.Random(n).getrandbits(8) for _ in range(n))
    assert oracle.sha1(m) == hashlib.sha1(m).digest()
    assert oracle.sha256(m) == hashlib.sha256(m).digest()
    assert oracle.sha384(m) == hashlib.sha384(m).digest()
    assert oracle.sha512(m) == hashlib.sha512(m).digest()
    assert oracle.md5(m) == hashlib.md5(m).digest()


def test_aes_fips197_appendix_c(oracle):
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    k128, k256 = bytes(range(16)), bytes(range(32))
    assert oracle.aes_encrypt_block(k128, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert oracle.aes_decrypt_block(k128, bytes.fromhex("69c4e0d86a7b0430d8cdb78070b4c55a")) == pt
    assert oracle.aes_encrypt_block(k256, pt).hex() == "8ea2b7ca516745bfeafc49904b496089"
    assert oracle.aes_decrypt_block(k256, bytes.fromhex("8ea2b7ca516745bfeafc49904b496089")) == pt


def test_rc4_rfc6229(oracle):
    # RFC 6229 section 2, key 0x0102030405 (40 bits) and 0x0102...10 (128 bits), keystream offset 0
    assert oracle.rc4(bytes.fromhex("0102030405"), bytes(16)).hex() == "b2396305f03dc027ccc3524a0a1118a8"
    assert oracle.rc4(bytes(range(1, 17)), bytes(16)).hex() == "9ac7cc9a609d1ef7b2932899cde41b97"


def test_pbkdf2_rfc6070(oracle):
    assert oracle.pbkdf2_hmac_sha1(b"password", b"salt", 1, 20).hex() == "0c60c80f961f0e71f3a9b524af6012062fe037a6"
    assert oracle.pbkdf2_hmac_sha1(b"password", b"salt", 4096, 20).hex() == "4b007901b765489abead49d926f721d065a429c1"
    assert oracle.pbkdf2_hmac_sha1(b"passwordPASSWORDpassword", b"saltSALTsaltSALTsaltSALTsaltSALTsalt", 4096,
                                   25).hex() == "3d2eec4fe41c849b80c8d83662c0e44a8b291a964cf2f07038"
    for it in (1, 2, 1024):
        pw, salt = os.urandom(32), os.urandom(16)
        assert oracle.pbkdf2_hmac_sha1(pw, salt, it, 32) == hashlib.pbkdf2_hmac("sha1", pw, salt, it, 32)


def test_bn_hex_decode_drops_leading_zero_bytes(oracle):
    # str_to_uchar (msoffcrypto_password_verifier.c:340-349): BN_bn2bin writes BN_num_bytes bytes
    assert oracle.bn_hex_decode("00ab12") == bytes.fromhex("ab12")
    assert oracle.bn_hex_decode("000ab1") == bytes.fromhex("0ab1")
    assert oracle.bn_hex_decode("abc") == bytes.fromhex("0abc")
    assert oracle.bn_hex_decode("0000") == b""
    assert oracle.bn_hex_decode("de40abf5") == bytes.fromhex("de40abf5")
    assert oracle.bn_hex_decode("12zz") == bytes.fromhex("12")
