"""The fd ends of the path: real read(2)/write(2).

Ingress: a peer thread writes base64 text into a pipe (or an AF_UNIX
socketpair) -> pipestream (ref src/pipestream.c:23-109) -> base64_decode
stage -> consumer.  Egress: a queuestream -> base64_encode stage ->
chunk_encode -> fdsink (the reference's tcp_connection egress loop,
src/tcp_connection.c:451-484, 669-727: 10,240-byte pulls) -> a pipe a peer
thread drains.  Every output is compared with the oracle (the reference's
decoder_read / the restated queuestream -> encoder -> chunkencoder stack).

CPU tests run the product's host C over the CPU stand-in for the device
(tests/csrc/libstage_fake.so, adversarial completion orders); GPU tests run
the product library on the MI355X.
"""
import numpy as np
import pytest

from oracle import pyoracle as orc
from tests import util


def _text(seed, n, kind):
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256, n, dtype=np.uint8)
    chars = orc.encode(raw)
    if kind == "crlf76":
        chars = b"\r\n".join(chars[i:i + 76] for i in range(0, len(chars), 76)) + b"\r\n"
    elif kind == "junk":
        a = np.frombuffer(chars, np.uint8)
        mask = rng.random(a.size) < 0.01
        chars = bytes(np.insert(a, np.nonzero(mask)[0], ord("!")).astype(np.uint8))
    return raw, chars


@pytest.fixture
def fake():
    L = util.fake_harness()
    yield L
    L.fake_configure(1, 0, 0)


@pytest.mark.parametrize("kind", ["clean", "crlf76", "junk"])
@pytest.mark.parametrize("sock", [False, True])
@pytest.mark.parametrize("write_chunk", [997, 1 << 16])
def test_fd_decode_fake(fake, kind, sock, write_chunk):
    """Short peer writes make the pipe run dry mid-stream (EAGAIN from
    read(2), the edge callback brings the consumer back); carries land at
    every block edge; the device completes out of order."""
    fake.fake_configure(11, 30, 0)
    raw, chars = _text(3, 600000, kind)
    got, err, _ = util.fd_decode(chars, write_chunk=write_chunk, read_size=4096, sock=sock,
                                 lib=fake)
    assert err == 0 and got is not None
    assert got.tobytes() == orc.decode(chars)
    assert got.tobytes() == raw.tobytes()


def test_fd_decode_empty_and_tiny(fake):
    for chars in (b"", b"Q", b"QU", b"QUI=", b"\r\n\r\n"):
        got, err, _ = util.fd_decode(chars, lib=fake)
        assert err == 0 and got.tobytes() == orc.decode(chars), chars


@pytest.mark.parametrize("max_chunk", [30, 4096, 1 << 20])
@pytest.mark.parametrize("sock", [False, True])
def test_fd_encode_fake(fake, max_chunk, sock):
    """The egress stack drained into a pipe by fdsink: framed bytes are the
    oracle stack's (same chunk sizes, so the encoder's read counts are the
    reference's), pieces spread over several queuestream elements."""
    fake.fake_configure(5, 30, 0)
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 300001, dtype=np.uint8).tobytes()
    pieces = [100000, 1, 2, 99998, 100000]
    got, err, _ = util.fd_encode(data, pieces, max_chunk=max_chunk, sock=sock, lib=fake)
    assert err == 0 and got is not None
    want = orc.chunked_encode(data, pieces, max_chunk=max_chunk, read_size=10240)
    assert got.tobytes() == want
    assert util.dechunk(got.tobytes()) == orc.encode(data)


@pytest.mark.parametrize("max_chunk", [4096, 1 << 20])
def test_fd_encode_fake_elements_past_the_arena_room(fake, max_chunk):
    """Queue elements far longer than a block's arena room (the GPU test's
    shapes): a block gathered by reading never takes more than its room
    (the fake's host buffers end at an inaccessible page, as pinned
    mappings do, so an overrun faults here)."""
    fake.fake_configure(7, 0, 0)
    rng = np.random.default_rng(23)
    data = rng.integers(0, 256, (16 << 20) + 1, dtype=np.uint8).tobytes()
    pieces = [1 << 20, 5, (15 << 20) - 4]
    got, err, _ = util.fd_encode(data, pieces, max_chunk=max_chunk, lib=fake)
    assert err == 0 and got is not None
    assert got.tobytes() == orc.chunked_encode(data, pieces, max_chunk=max_chunk,
                                               read_size=10240)


@pytest.mark.parametrize("sock", [False, True])
def test_fd_encode_fake_unframed(fake, sock):
    """fdsink reading the encoder itself (no chunk stage, so no lending):
    its copying read path, 10,240-byte pulls, into a pipe or socket."""
    fake.fake_configure(3, 30, 0)
    rng = np.random.default_rng(31)
    data = rng.integers(0, 256, 700003, dtype=np.uint8).tobytes()
    pieces = [1, 350000, 4, 349998]
    for pos62, pos63, pad in ((-1, -1, True), ("-", "_", False)):
        got, err, _ = util.fd_encode(data, pieces, max_chunk=0, pos62=pos62, pos63=pos63,
                                     pad=pad, sock=sock, lib=fake)
        assert err == 0 and got is not None
        assert got.tobytes() == orc.encode(data, pos62=pos62, pos63=pos63, pad=pad)


def test_fd_encode_empty(fake):
    got, err, _ = util.fd_encode(b"", lib=fake)
    assert err == 0 and got.tobytes() == orc.chunked_encode(b"", max_chunk=1 << 20,
                                                            read_size=10240)


@pytest.mark.parametrize("what", ["minus_one", "regular_file"])
def test_fdsink_unwatchable_fd_calls_back(fake, tmp_path, what):
    """fdsink over a descriptor the loop cannot watch (-1; a regular file,
    which epoll refuses): the sink ends with the error, reported from the
    loop, so a callback registered after open_fdsink() returned is still
    performed (it used to be marked done at once and the
    callback never ran)."""
    import ctypes
    import errno
    import os
    fd = -1
    if what == "regular_file":
        fd = os.open(str(tmp_path / "sink.bin"), os.O_WRONLY | os.O_CREAT)
    err = ctypes.c_int(0)
    fired = fake.h_fdsink_unwatchable(fd, ctypes.byref(err))
    assert fired == 1
    assert err.value in (errno.EBADF, errno.EPERM), err.value
    if what == "regular_file":  # the sink owned and closed it
        with pytest.raises(OSError):
            os.fstat(fd)


def test_fd_ends_leak_check(fake):
    """The reference runner's counting allocator (test/asynctest.c:111-147)
    around both fd ends: pipestream, fdsink, stages, hub -- nothing left."""
    raw, chars = _text(4, 200000, "crlf76")
    (got, err, _), left = util.counted(util.fd_decode, chars, read_size=1000, lib=fake)
    assert err == 0 and got.tobytes() == raw.tobytes() and left == 0
    (got, err, _), left = util.counted(util.fd_encode, raw.tobytes(), lib=fake)
    assert err == 0 and left == 0
    assert util.dechunk(got.tobytes()) == chars.replace(b"\r\n", b"")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["clean", "crlf76", "junk"])
@pytest.mark.parametrize("sock", [False, True])
def test_fd_decode_gpu(kind, sock):
    raw, chars = _text(21, 24 << 20, kind)
    got, err, _ = util.fd_decode(chars, write_chunk=1 << 20, read_size=1 << 18, sock=sock)
    assert err == 0 and got is not None
    assert got.tobytes() == raw.tobytes()
    assert got.size == len(orc.decode(chars))


@pytest.mark.gpu
def test_fd_decode_gpu_short_writes():
    raw, chars = _text(22, 3 << 20, "crlf76")
    got, err, _ = util.fd_decode(chars, write_chunk=4093, read_size=1000)
    assert err == 0 and got.tobytes() == raw.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("max_chunk", [4096, 1 << 20])
def test_fd_encode_gpu(max_chunk):
    rng = np.random.default_rng(23)
    data = rng.integers(0, 256, (16 << 20) + 1, dtype=np.uint8).tobytes()
    pieces = [1 << 20, 5, (15 << 20) - 4]
    got, err, _ = util.fd_encode(data, pieces, max_chunk=max_chunk)
    assert err == 0 and got is not None
    assert got.tobytes() == orc.chunked_encode(data, pieces, max_chunk=max_chunk,
                                               read_size=10240)


@pytest.mark.gpu
def test_fd_encode_gpu_unframed():
    rng = np.random.default_rng(29)
    data = rng.integers(0, 256, (8 << 20) + 2, dtype=np.uint8).tobytes()
    got, err, _ = util.fd_encode(data, [1 << 20, (7 << 20) + 2], max_chunk=0, sock=True)
    assert err == 0 and got is not None
    assert got.tobytes() == orc.encode(data)
