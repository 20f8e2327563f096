"""Restatement of Spacedrive's content-addressing functions -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may
import this module, and only as the checker; the product never does.

* ``generate_cas_id``  follows ``/root/reference/core/src/object/cas.rs:23-62``
  (constants ``cas.rs:10-15``).
* ``file_checksum``    follows ``/root/reference/core/src/object/validation/hash.rs:10-24``.
* ``cas_message``      is the exact byte stream ``generate_cas_id`` feeds to
  ``Hasher::update`` -- the same stream the product's stager writes into the staged
  buffer (``include/sd_cas.h``, ``sd_cas_stage_plan``).
* ``synth_*``          is the counter-based synthetic file-content generator of
  ``SURVEY.md`` §8(d), shared bit-for-bit with ``oracle/sd_oracle.c`` and the device
  generator ``spacedrive_amd/csrc/synth.hip``.
"""

from __future__ import annotations

import struct

import numpy as np

try:  # package-relative when imported as oracle.cas_spec, flat when run from oracle/
    from .blake3_spec import Hasher, blake3
except ImportError:  # pragma: no cover
    from blake3_spec import Hasher, blake3

# cas.rs:10-15
SAMPLE_COUNT = 4
SAMPLE_SIZE = 1024 * 10
HEADER_OR_FOOTER_SIZE = 1024 * 8
MINIMUM_FILE_SIZE = 1024 * 100
# cas.rs:18,21 (const_assert!)
assert HEADER_OR_FOOTER_SIZE * 2 + SAMPLE_COUNT * SAMPLE_SIZE < MINIMUM_FILE_SIZE
assert SAMPLE_SIZE > HEADER_OR_FOOTER_SIZE

SAMPLED_MSG_LEN = 8 + 2 * HEADER_OR_FOOTER_SIZE + SAMPLE_COUNT * SAMPLE_SIZE  # 57352

# hash.rs:8
CHECKSUM_READ_LEN = 1048576


def sample_windows(size: int) -> list:
    """(offset, length) windows read by the sampled branch, in hashing order.

    Traces cas.rs:31-58 literally: ``current_pos`` starts at the 8192 returned by the
    header ``read_exact`` (:35-37); each loop iteration reads SAMPLE_SIZE at
    ``current_pos`` (:43) and breaks once ``current_pos >= 8192 + 3*seek_jump`` (:46),
    otherwise seeks to ``current_pos + seek_jump`` (:50); then the footer (:54-58).
    """
    assert size > MINIMUM_FILE_SIZE
    wins = [(0, HEADER_OR_FOOTER_SIZE)]
    current_pos = HEADER_OR_FOOTER_SIZE
    seek_jump = (size - HEADER_OR_FOOTER_SIZE * 2) // SAMPLE_COUNT  # :41
    while True:
        wins.append((current_pos, SAMPLE_SIZE))
        if current_pos >= HEADER_OR_FOOTER_SIZE + seek_jump * (SAMPLE_COUNT - 1):
            break
        current_pos = current_pos + seek_jump
    wins.append((size - HEADER_OR_FOOTER_SIZE, HEADER_OR_FOOTER_SIZE))
    return wins


def cas_message(read_at, size: int) -> bytes:
    """Exact hashed stream of generate_cas_id for a file whose length is ``size``;
    ``read_at(off, n)`` returns file bytes.  (``cas_message_file`` covers a file whose
    length differs from ``size``.)"""
    head = struct.pack("<Q", size)  # cas.rs:25 (little-endian u64)
    if size <= MINIMUM_FILE_SIZE:  # cas.rs:27 -- note <=, 102400 is hashed whole
        return head + read_at(0, size)
    return head + b"".join(read_at(o, n) for o, n in sample_windows(size))


class UnexpectedEof(EOFError):
    """read_exact hit the end of the file: io::ErrorKind::UnexpectedEof (cas.rs:36,43,56)."""


def cas_message_file(content: bytes, size: int) -> bytes:
    """generate_cas_id's hashed stream for a file holding ``content`` when the caller passes
    ``size`` (metadata that may be stale: the two lengths may differ).

    * ``size <= 102400`` (cas.rs:27-29): ``fs::read`` hashes every byte the file holds,
      however many there are -- ``le64(size) || content``.
    * else (cas.rs:31-58): each ``read_exact`` at the traced position raises
      UnexpectedEof when the file ends inside its window; the seeks never fail forward
      (a seek past EOF is legal, the read after it fails); the footer is read at
      ``SeekFrom::End(-8192)`` -- the file's real end -- which fails with EINVAL
      (OSError) when the file is shorter than 8192 bytes.
    """
    import errno

    head = struct.pack("<Q", size)
    if size <= MINIMUM_FILE_SIZE:
        return head + content
    wins = sample_windows(size)[:-1]
    out = [head]
    for off, n in wins:  # header (:35-38) and the samples (:42-51)
        if off + n > len(content):
            raise UnexpectedEof(f"read_exact of {n} bytes at {off} past EOF {len(content)}")
        out.append(content[off:off + n])
    end = len(content) - HEADER_OR_FOOTER_SIZE  # :54 seek(End(-8192))
    if end < 0:
        raise OSError(errno.EINVAL, "invalid seek to a negative position")
    out.append(content[end:end + HEADER_OR_FOOTER_SIZE])  # :56-58 (always whole here)
    return b"".join(out)


def generate_cas_id_file(content: bytes, size: int) -> str:
    """cas.rs:23-62 on a file holding ``content``, called with ``size`` (see cas_message_file)."""
    return Hasher().update(cas_message_file(content, size)).finalize().hex()[:16]


def generate_cas_id(read_at, size: int) -> str:
    """cas.rs:23-62 -> 16 lowercase hex chars (first 8 bytes of the BLAKE3 hash)."""
    h = Hasher().update(cas_message(read_at, size)).finalize()
    return h.hex()[:16]  # cas.rs:61


def generate_cas_id_bytes(content: bytes) -> str:
    return generate_cas_id(lambda o, n: content[o:o + n], len(content))


def file_checksum(content: bytes) -> str:
    """hash.rs:10-24: 1 MiB reads until a short read; output is the full 64-hex hash.

    BLAKE3 output is independent of update split points, so the read loop reduces to
    one hash of the whole content; the loop is kept to mirror the reference.
    """
    pos = 0

    def read(n):
        nonlocal pos
        buf = content[pos:pos + n]
        pos += len(buf)
        return buf

    return file_checksum_reads(read)


def file_checksum_reads(read) -> str:
    """hash.rs:14-20 over a reader: ``read(n)`` is one read call returning up to n bytes
    (tokio's ``File::read`` issues one ``read`` per call).  Every returned byte is hashed;
    the loop ends at the first call that returns fewer than BLOCK_LEN bytes -- the end of
    a regular file, or simply a short read of a pipe."""
    h = Hasher()
    while True:
        buf = read(CHECKSUM_READ_LEN)
        h.update(buf)
        if len(buf) != CHECKSUM_READ_LEN:
            break
    return h.finalize().hex()


# ---------------------------------------------------------------- synthetic content
SYNTH_SEED = 0x5D5DCA51D
GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
TWIN_OFFSET = HEADER_OR_FOOTER_SIZE + SAMPLE_SIZE  # 18432: never inside a sample window


def splitmix64(x):
    """splitmix64 finaliser on uint64 numpy arrays (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_bytes(content_id: int, twin: int, offset: int, length: int) -> bytes:
    """Bytes [offset, offset+length) of synthetic content ``content_id``.

    byte o = byte (o & 7) (little-endian) of splitmix64(SEED ^ (cid*GOLDEN) ^ (o >> 3));
    a "sample twin" (twin != 0) additionally XORs byte TWIN_OFFSET with (twin & 0xFF) | 1,
    so its cas_id equals the original's while its checksum differs.
    """
    if length <= 0:
        return b""
    w0 = offset >> 3
    w1 = (offset + length + 7) >> 3
    key = (SYNTH_SEED ^ ((content_id * GOLDEN) & M64)) & M64
    words = splitmix64(np.uint64(key) ^ np.arange(w0, w1, dtype=np.uint64))
    raw = words.astype("<u8").tobytes()
    start = offset - (w0 << 3)
    out = bytearray(raw[start:start + length])
    if twin and offset <= TWIN_OFFSET < offset + length:
        out[TWIN_OFFSET - offset] ^= (twin & 0xFF) | 1
    return bytes(out)


def synth_reader(content_id: int, twin: int = 0):
    return lambda o, n: synth_bytes(content_id, twin, o, n)
