"""The C-ABI library loads and exports every declared symbol; host-only
logic (loop, streams, stage error paths) works without a GPU.  CPU only:
nothing here launches a kernel."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from async_amd import _lib
from tests import util

ROOT = util.ROOT


def _declared(header: str):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"static inline[^{]*\{[^}]*\}", "", src)
    # file-scope declarations start in column 0: "<type> [*]name(".
    return set(re.findall(r"(?m)^(?:const\s+)?[a-z_]\w*[\s*]+([a-z_]\w*)\s*\(", src)) \
        - {"void"}


def _exported():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_built_in_tree():
    assert os.path.exists(_lib.LIB_PATH), "run make / __graft_entry__.build()"


def test_every_declared_symbol_is_exported():
    exported = _exported()
    headers = ["b64x.h", "base64encoder.h", "base64decoder.h", "async.h",
               "bytestream_1.h", "blobstream.h", "nicestream.h", "fsalloc.h"]
    for h in headers:
        for name in _declared(h):
            assert name in exported, f"{h}: {name} not exported"
    assert "NULL_ACTION_1" in exported
    # and the Python binding covers all of b64x.h
    assert _declared("b64x.h") == set(_lib.SIGNATURES)
    for name in _lib.STAGE_SYMBOLS:
        assert name in exported, name


def test_product_has_no_variant_knobs():
    """The product libraries carry no kernel-variant or test hooks and read
    no tuning variable that could select another kernel form: the only
    knobs a user has are the documented ones, none of which
    changes the bytes produced."""
    core = os.path.join(ROOT, "async_amd", "libasync_b64_core.so")
    for path in (_lib.LIB_PATH, core):
        out = subprocess.run(["nm", "-D", "--defined-only", path],
                             capture_output=True, text=True, check=True).stdout
        assert "b64x__" not in out, path
        blob = open(path, "rb").read()
        assert b"ASYNC_B64_TUNE" not in blob, path
    hooks = subprocess.run(["nm", "-D", "--defined-only", util.HOOKS],
                           capture_output=True, text=True, check=True).stdout
    assert "b64x__test_range_chunks" in hooks


def test_kernel_barriers_wait_for_lds():
    """Every barrier in the kernels is block_sync() (an explicit
    s_waitcnt lgkmcnt(0), then __syncthreads()): hipcc's barrier at the top
    of the held suffix kernel's loop did not wait for thread 0's LDS write of
    the next ticket, and a wave now and then decoded another tile (DESIGN.md
    §5)."""
    import re
    src = open(os.path.join(ROOT, "async_amd", "csrc", "b64x_kernels.hip")).read()
    code = re.sub(r"//[^\n]*", "", src)
    a = code.index("DEV void block_sync()")
    b = code.index("}", a) + 1
    assert "s_waitcnt lgkmcnt(0)" in code[a:b] and "__syncthreads()" in code[a:b]
    assert "__syncthreads()" not in code[:a] + code[b:]


def _isa():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "tools"))
    import isa_check
    return isa_check, isa_check.disassemble(_lib.LIB_PATH)


# The kernels the product launches (b64x_kernels.hip); nothing else may be in
# its code object: no A/B variant, no experiment, no test hook.
SHIPPED_KERNELS = {
    "k_encode", "k_encode_flat", "k_encode_tight2<2>", "k_encode_strided<2, true>",
    "k_encode_ragged",
    "k_decode_probe", "k_decode_lines<false>", "k_decode_lines<true>",
    "k_decode_suffix_held<false, false>", "k_decode_suffix_held<true, false>",
    "k_decode_suffix_held<false, true>", "k_decode_suffix_held<true, true>",
    "k_decode_pass1<2, true>", "k_decode_scan2",
    "k_decode_pass2d",
    "k_decode_slots<2>", "k_rows_prep", "k_decode_rows_lines<4, false>",
    "k_decode_rows_lines<4, true>", "k_rows_finish", "k_decode_batch_fast<false>",
    "k_decode_batch_fast<true>", "k_decode_batch_fix2<false>", "k_decode_batch_fix2<true>",
    "k_batch_finish",
    "k_result_zero", "k_stamp", "k_spell_head", "k_gather_host", "k_fill_splitmix64",
}


def test_code_object_holds_only_shipped_kernels():
    """the experiments (the count-ahead suffix kernel, the
    tile-shape knobs) are out of the product translation unit; the code
    object's kernel symbols are exactly the kernels the library launches."""
    isa, dis = _isa()
    names = subprocess.run(["c++filt"], input="\n".join(sorted(isa.kernel_symbols(dis))),
                           capture_output=True, text=True, check=True).stdout.split("\n")
    got = set()
    for n in names:
        if not n:
            continue
        m = re.match(r"^(?:void )?(?:\(anonymous namespace\)::)?([\w]+(?:<[^>]*>)?)\(", n)
        got.add(m.group(1) if m else n)
    assert got == SHIPPED_KERNELS, (got - SHIPPED_KERNELS, SHIPPED_KERNELS - got)


def test_code_object_barriers_drain_lds():
    """On gfx950 the hardware barrier does not wait for LDS writes, and the
    compiler may drop the soft lgkmcnt(0) that __syncthreads()'s fence leaves
    before it (it did at k_decode_suffix_held's loop header in round 5:
    profiles/r06_isa_barrier_evidence.txt).  Over the control-flow graph of
    every kernel in the shipped code object, no s_barrier is reached with an
    LDS write or a global -> LDS copy in flight; and in the kernels that copy
    into LDS, the LDS reads reached while a copy may be in flight are only the
    decode's other tables and window (the byte lookups, the compaction
    selectors, the held window dwords): the copies' buffers are read as whole
    16-byte rows (ds_read_b128), after the reader's own vmcnt(0)."""
    isa, dis = _isa()
    assert isa.barrier_count(dis) > 20
    assert isa.barrier_report(dis) == []
    reads = isa.dma_reads(dis)
    assert reads, "k_decode_suffix_held copies its ranges into LDS"
    allowed = {"ds_read_u8", "ds_read_b32", "ds_read2_b32", "ds_read2st64_b32"}
    for name, rows in reads.items():
        kinds = {t.split()[0] for _, t in rows}
        assert kinds <= allowed, (name, kinds - allowed)


def test_isa_check_finds_the_round5_race():
    """The checker flags the pattern it is meant to catch: a loop whose
    header barrier has no wait while its back edge carries an LDS write
    (a hand-written listing in the disassembler's format)."""
    sys_path = os.path.join(ROOT, "tests", "tools")
    import sys
    sys.path.insert(0, sys_path)
    import isa_check
    def listing(wait):
        rows = ["0000000000001000 <k>:",
                "\tv_mov_b32_e32 v2, 0 // 000000001000: 0",
                "\tds_write_b32 v2, v1 offset:64 // 000000001004: 0",
                "\ts_waitcnt lgkmcnt(0) // 000000001008: 0",
                "\ts_barrier // 00000000100C: 0",
                "\tv_lshlrev_b32_e32 v3, 2, v61 // 000000001010: 0"]
        if wait:
            rows.append("\ts_waitcnt lgkmcnt(0) // 000000001014: 0")
        else:
            rows.append("\ts_nop 0 // 000000001014: 0")
        rows += ["\ts_barrier // 000000001018: 0",
                 "\tds_read_b32 v3, v3 offset:64 // 00000000101C: 0",
                 "\ts_waitcnt lgkmcnt(0) // 000000001020: 0",
                 "\tds_write_b32 v6, v4 offset:64 // 000000001024: 0",
                 "\ts_cbranch_vccz 1 // 000000001028: 0 <k+0x30>",
                 "\ts_branch 65528 // 00000000102C: 0 <k+0x10>",
                 "\ts_endpgm // 000000001030: 0"]
        return "\n".join(rows)
    assert isa_check.barrier_report(listing(True)) == []
    bad = isa_check.barrier_report(listing(False))
    assert [(r[1], r[2]) for r in bad] == [(0x18, "lds")]


def test_bind_thread_without_a_gpu_leaves_the_thread():
    """b64x_bind_thread (and the hub's call of it) is a no-op that reports an
    error when there is no device: the thread's CPU mask is unchanged."""
    import threading
    lib = _lib.load()
    out = {}

    def run():
        before = os.sched_getaffinity(0)
        out["rc"] = lib.b64x_bind_thread(-1)
        out["same"] = os.sched_getaffinity(0) == before
        out["node"] = lib.b64x_device_numa_node(-1)
    t = threading.Thread(target=run)
    t.start()
    t.join()
    assert out["rc"] < 0 and out["same"] and out["node"] < 0


def test_placement_helpers():
    from async_amd import placement as pl
    assert pl.parse_cpulist("0-3,7,9-10") == {0, 1, 2, 3, 7, 9, 10}
    assert pl.cpulist({0, 1, 2, 3, 7, 9, 10}) == "0-3,7,9-10"
    cpus = os.sched_getaffinity(0)
    assert pl.cpu_node(min(cpus)) >= 0 or not os.path.isdir("/sys/devices/system/node/node0")
    assert isinstance(pl.pages_by_node(1 << 20), dict)


def test_every_environment_knob_is_documented():
    """Every ASYNC_B64_* variable the product libraries can read is in
    INTEGRATION.md's runtime-configuration table."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    core = os.path.join(ROOT, "async_amd", "libasync_b64_core.so")
    for path in (_lib.LIB_PATH, core):
        names = set(re.findall(rb"ASYNC_B64_[A-Z0-9_]+", open(path, "rb").read()))
        assert names, path
        for n in names:
            assert f"`{n.decode()}`" in doc, (path, n)


def test_binding_loads_and_sizes():
    lib = _lib.load()
    assert lib.b64x_encoded_len(0, True) == 0
    assert lib.b64x_encoded_len(1, True) == 4 and lib.b64x_encoded_len(1, False) == 2
    assert lib.b64x_encoded_len(2, False) == 3 and lib.b64x_encoded_len(3, False) == 4
    assert lib.b64x_encoded_len(1 << 30, True) == 1431655768
    assert lib.b64x_decoded_cap(1431655768) == 1073741826
    assert lib.b64x_decode_workspace_size(1 << 30) > 0
    assert b"gfx950" in lib.b64x_build_info()
    assert lib.b64x_strerror(-22) == b"invalid argument"


def test_no_gpu_fails_loudly():
    """Without a usable gfx950 the ABI reports ENODEV; it never computes on
    the CPU instead."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _lib.load()
    assert lib.b64x_device_check() == -19
    buf = (ctypes.c_uint8 * 16)()
    a = _lib.alphabet()
    assert lib.b64x_encode_dev(ctypes.addressof(buf), 3, ctypes.addressof(buf),
                               ctypes.byref(a), None) == -19
    assert lib.b64x_session_open(1024) is None
    # the bytestream_1 stages surface it as -1 / errno ENODEV on read()
    out, err = util.stage_encode(b"hello world")
    assert out is None and err == 19
    out, err = util.stage_decode(b"aGVsbG8=")
    assert out is None and err == 19


def test_argument_validation():
    lib = _lib.load()
    a = _lib.alphabet()
    assert lib.b64x_encode_dev(None, 5, None, ctypes.byref(a), None) == -22
    assert lib.b64x_encode_dev(None, 0, None, ctypes.byref(a), None) == 0
    assert lib.b64x_decode_dev(None, 4, None, None, ctypes.byref(a), 0, None, None) == -22
    res = _lib.DecResult()
    assert lib.b64x_decode_dev(None, 4, None, ctypes.byref(res), ctypes.byref(a),
                               0x80, None, None) == -22


@pytest.mark.parametrize("burst", [0, 1, 7, 113])
@pytest.mark.parametrize("read_size", [1, 3, 200, 4096])
def test_loop_and_streams_copy(burst, read_size):
    """blobstream -> nicestream -> consumer on the product event loop: bytes
    arrive intact and nicestream's EAGAIN/retry path is exercised."""
    rng = np.random.default_rng(burst * 7 + read_size)
    data = rng.integers(0, 256, 5000, dtype=np.uint8)
    out = np.empty(6000, np.uint8)
    err = ctypes.c_int(0)
    eag = ctypes.c_size_t(0)
    n = util.harness().h_copy_stream(data.ctypes.data, data.size, burst, read_size,
                                     out.ctypes.data, out.size, ctypes.byref(err),
                                     ctypes.byref(eag))
    assert n == data.size and err.value == 0
    assert (out[:n] == data).all()
    if burst:
        assert eag.value > 0


def test_async_register_is_edge_triggered():
    """async_register() keeps the reference's contract (include/async.h,
    src/async.c:733-760): the descriptor becomes non-blocking, and the action
    runs on a change of state -- once per write here -- not again while
    unread input is merely pending (level-triggered delivery would call it on
    every loop turn)."""
    L = _lib.load()

    class Action(ctypes.Structure):
        _fields_ = [("obj", ctypes.c_void_p), ("act", ctypes.c_void_p)]

    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    L.make_async.restype = ctypes.c_void_p
    L.async_now.argtypes = [ctypes.c_void_p]
    L.async_now.restype = ctypes.c_uint64
    L.async_register.argtypes = [ctypes.c_void_p, ctypes.c_int, Action]
    L.async_unregister.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.async_timer_start.argtypes = [ctypes.c_void_p, ctypes.c_uint64, Action]
    L.async_timer_start.restype = ctypes.c_void_p
    L.async_loop.argtypes = [ctypes.c_void_p]
    L.async_quit_loop.argtypes = [ctypes.c_void_p]
    L.destroy_async.argtypes = [ctypes.c_void_p]
    async_ = L.make_async()
    calls = []
    on_fd = CB(lambda obj: calls.append(1))
    on_quit = CB(lambda obj: L.async_quit_loop(async_))
    quit_addr = ctypes.cast(on_quit, ctypes.c_void_p).value

    def turn(ms=30):
        before = len(calls)
        L.async_timer_start(async_, L.async_now(async_) + ms * 1000000,
                            Action(None, quit_addr))
        assert L.async_loop(async_) == 0
        return len(calls) - before

    r, w = os.pipe()
    try:
        assert os.get_blocking(r)
        assert L.async_register(async_, r, Action(None, ctypes.cast(on_fd, ctypes.c_void_p).value)) == 0
        assert not os.get_blocking(r)
        turn()                      # a registration may bring one spurious call
        os.write(w, b"x")
        assert turn() == 1          # one edge, one call
        assert turn() == 0          # still unread: no further call (edge-triggered)
        os.write(w, b"y")
        assert turn() == 1
        assert os.read(r, 16) == b"xy"
        assert L.async_unregister(async_, r) == 0
    finally:
        os.close(r)
        os.close(w)
        L.destroy_async(async_)


def test_core_library_dependencies():
    """The stages-only library (INTEGRATION.md Option A) needs exactly the
    documented host-library symbols besides libc/HIP."""
    core = os.path.join(ROOT, "async_amd", "libasync_b64_core.so")
    out = subprocess.run(["nm", "-D", "--undefined-only", core],
                         capture_output=True, text=True, check=True).stdout
    # every unversioned symbol that is not the HIP runtime's or a compiler
    # hook must be one of the documented host-library names
    names = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    ours = {n for n in names if "@" not in n and not n.startswith(("_", "hip"))}
    assert ours == {"async_wound", "async_execute", "async_register", "async_unregister",
                    "NULL_ACTION_1", "fsalloc", "fscalloc", "fsfree"}
    # the allocator is the reference's (fsdyn's) in a reference build: the
    # core library must not bring its own
    defined = subprocess.run(["nm", "-D", "--defined-only", core],
                             capture_output=True, text=True, check=True).stdout
    assert not re.search(r"\bfs(alloc|calloc|free)\b", defined)
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for n in ours:
        assert f"`{n}" in doc, n


def test_edges_arriving_after_quit_are_kept():
    """Two descriptors become readable in the same poll; the action of the
    first one quits the loop.  The second edge is not dropped (an
    edge-triggered registration would never report it again): it is
    delivered when the loop runs again, as the reference's loop delivers
    every triggered event (src/async.c:300-330)."""
    L = _lib.load()

    class Action(ctypes.Structure):
        _fields_ = [("obj", ctypes.c_void_p), ("act", ctypes.c_void_p)]

    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    L.make_async.restype = ctypes.c_void_p
    L.async_now.argtypes = [ctypes.c_void_p]
    L.async_now.restype = ctypes.c_uint64
    L.async_register.argtypes = [ctypes.c_void_p, ctypes.c_int, Action]
    L.async_unregister.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.async_timer_start.argtypes = [ctypes.c_void_p, ctypes.c_uint64, Action]
    L.async_timer_start.restype = ctypes.c_void_p
    L.async_loop.argtypes = [ctypes.c_void_p]
    L.async_quit_loop.argtypes = [ctypes.c_void_p]
    L.destroy_async.argtypes = [ctypes.c_void_p]
    async_ = L.make_async()
    calls = []
    on_fd = CB(lambda obj: (calls.append(obj), L.async_quit_loop(async_)))
    on_quit = CB(lambda obj: L.async_quit_loop(async_))
    quit_addr = ctypes.cast(on_quit, ctypes.c_void_p).value
    fd_addr = ctypes.cast(on_fd, ctypes.c_void_p).value
    p1, p2 = os.pipe(), os.pipe()
    try:
        assert L.async_register(async_, p1[0], Action(1, fd_addr)) == 0
        assert L.async_register(async_, p2[0], Action(2, fd_addr)) == 0
        L.async_timer_start(async_, L.async_now(async_) + 30 * 1000000, Action(None, quit_addr))
        assert L.async_loop(async_) == 0   # spurious registration calls, if any
        calls.clear()
        os.write(p1[1], b"x")
        os.write(p2[1], b"y")
        assert L.async_loop(async_) == 0   # the first action quits
        assert len(calls) == 1
        L.async_timer_start(async_, L.async_now(async_) + 30 * 1000000, Action(None, quit_addr))
        assert L.async_loop(async_) == 0
        assert sorted(calls) == [1, 2]
        assert L.async_unregister(async_, p1[0]) == 0
        assert L.async_unregister(async_, p2[0]) == 0
    finally:
        for a, b in (p1, p2):
            os.close(a)
            os.close(b)
        L.destroy_async(async_)
