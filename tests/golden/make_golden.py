"""Regenerates the golden fixtures in tests/golden/ from the pure-Python spec oracle.

    python tests/golden/make_golden.py

Inputs are deterministic: the official BLAKE3 test-vector pattern (byte i = i % 251)
and the counter-based synthetic generator of SURVEY.md §8(d) (oracle/cas_spec.py).
The reference's own fixtures are recorded verbatim where they exist: the BLAKE3 KAT
``DERIVE_B3_EXPECTED`` (/root/reference/crates/crypto/src/keys/hashing.rs:210-213, inputs
:121,132-141, material = key || salt per crates/crypto/src/types.rs:164-166).  The
reference's hot path (cas.rs / hash.rs) has no tests of its own, so the
cas_id / checksum goldens below are oracle outputs, pinned indirectly through the KAT
and the official BLAKE3 vectors that the same oracle reproduces.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import blake3_spec as b3  # noqa: E402
from oracle import cas_spec as cs  # noqa: E402

# Official BLAKE3 test vectors (test_vectors.json of the BLAKE3 spec repository,
# input = bytes(i % 251 for i in range(len)), first 32 bytes of the hash).  Recorded
# as published; the oracle must reproduce each one.
OFFICIAL = {
    0: "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    1: "2d3adedff11b61f14c886e35afa036736dcd87a74d27b5c1510225d0f592e213",
    1023: "10108970eeda3eb932baac1428c7a2163b0e924c9a9e25b35bba72b28f70bd11",
    1024: "42214739f095a406f3fc83deb889744ac00df831c10daa55189b5d121c855af7",
    1025: "d00278ae47eb27b34faecf67b4fe263f82d5412916c1ffd97c8cb7fb814b8444",
    2048: "e776b6028c7cd22a4d0ba182a8bf62205d2ef576467e838ed6f2529b85fba24a",
    2049: "5f4d72f40d7a5f82b15ca2b2e44b1de3c2ef86c426c95c1af0b6879522563030",
    3072: "b98cb0ff3623be03326b373de6b9095218513e64f1ee2edd2525c7ad1e5cffd2",
    3073: "7124b49501012f81cc7f11ca069ec9226cecb8a2c850cfe644e327d22d3e1cd3",
    4096: "015094013f57a5277b59d8475c0501042c0b642e531b0a1c8f58d2163229e969",
    4097: "9b4052b38f1c5fc8b1f9ff7ac7b27cd242487b3d890d15c96a1c25b8aa0fb995",
    5120: "9cadc15fed8b5d854562b26a9536d9707cadeda9b143978f319ab34230535833",
    8192: "aae792484c8efe4f19e2ca7d371d8c467ffb10748d8a5a1ae579948f718a2a63",
    8193: "bab6c09cb8ce8cf459261398d2e7aef35700bf488116ceb94a36d0f5f1b7bc3b",
    16384: "f875d6646de28985646f34ee13be9a576fd515f76b5b0a26bb324735041ddde4",
    31744: "62b6960e1a44bcc1eb1a611a8d6235b6b4b78f32e7abc4fb4c6cdcce94895c47",
    102400: "bc3e3d41a1146b069abffad3c0d44860cf664390afce4d9661f7902e7943e085",
}

# crates/crypto/src/keys/hashing.rs:121 (context), :132-141 (KEY, SALT), :210-213 (expected)
KAT_DERIVE_B3 = {
    "context": "spacedrive 2023-02-09 17:44:14 test key derivation",
    "key_hex": "23" * 32,
    "salt_hex": "ff" * 16,
    "expected": [27, 34, 251, 101, 201, 89, 78, 90, 20, 175, 62, 206, 200, 153, 166, 103,
                 118, 179, 194, 44, 216, 26, 48, 120, 137, 157, 60, 234, 234, 53, 46, 60],
    "source": "crates/crypto/src/keys/hashing.rs:210-213,323-328",
}

# SURVEY.md §8(d) edge sizes: block (64 B), chunk (1 KiB incl. the 8-byte size header),
# the sample threshold (102400 hashed whole, 102401 sampled) and hash.rs's 1 MiB reads.
EDGE_SIZES = [0, 1, 55, 56, 57, 63, 64, 65, 1015, 1016, 1017, 2040, 2041, 16376, 16377,
              65536, 102399, 102400, 102401, 131072, (1 << 20) - 1, 1 << 20, (1 << 20) + 1,
              (1 << 32) + 1]
CHECKSUM_SIZES = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3072, 3073, 7168, 8193,
                  65536, 102400, 102401, (1 << 20) - 1, 1 << 20, (1 << 20) + 1]


def pattern_reader(o: int, n: int) -> bytes:
    return bytes((o + k) % 251 for k in range(n))


def main() -> None:
    pat = lambda n: pattern_reader(0, n)  # noqa: E731
    blake = {}
    for n, expected in OFFICIAL.items():
        got = b3.blake3(pat(n)).hex()
        assert got == expected, (n, got, expected)
        blake[str(n)] = expected
    kat = dict(KAT_DERIVE_B3)
    got = list(b3.derive_key(kat["context"], bytes.fromhex(kat["key_hex"] + kat["salt_hex"])))
    assert got == kat["expected"]

    cas_pattern = {str(s): cs.generate_cas_id(pattern_reader, s) for s in EDGE_SIZES}
    cas_synth = []
    for i, s in enumerate(EDGE_SIZES):
        for twin in (0, 3):
            if twin and s <= cs.MINIMUM_FILE_SIZE:
                continue
            cas_synth.append({"size": s, "content_id": 1000 + i, "twin": twin,
                              "cas_id": cs.generate_cas_id(cs.synth_reader(1000 + i, twin), s)})
    checks_pattern = {str(s): cs.file_checksum(pat(s)) for s in CHECKSUM_SIZES}
    checks_synth = []
    for i, s in enumerate(CHECKSUM_SIZES):
        for twin in (0, 3):
            if twin and s <= cs.TWIN_OFFSET:
                continue
            checks_synth.append({"size": s, "content_id": 2000 + i, "twin": twin,
                                 "checksum": cs.file_checksum(cs.synth_bytes(2000 + i, twin, 0, s))})
    synth_prefix = {str(c): cs.synth_bytes(c, 0, 0, 40).hex() for c in (0, 1, 12345, (1 << 40) + 7)}

    out = {
        "blake3_official.json": {"pattern": "byte i = i % 251", "hash": blake},
        "kat_derive_b3.json": kat,
        "cas_pattern.json": {"pattern": "byte i = i % 251", "cas_id": cas_pattern},
        "cas_synth.json": {"generator": "SURVEY.md 8(d) splitmix64, seed 0x5D5DCA51D",
                           "files": cas_synth, "synth_prefix40": synth_prefix},
        "checksum_pattern.json": {"pattern": "byte i = i % 251", "checksum": checks_pattern},
        "checksum_synth.json": {"files": checks_synth},
    }
    for name, obj in out.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
