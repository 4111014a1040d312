"""Replay format, ring linearisation (__copy_buffer) and the generator."""
import os

import numpy as np
import pytest

from numamma_amd.replay import (RECORD_BYTES, Buffer, Replay, SynthConfig, flatten_insertions,
                                generate)


def test_roundtrip(tmp_path):
    rp = generate(SynthConfig(nb_samples=20_000, nb_intervals=300, lost_frac=1e-3, wrap_one=True, seed=3))
    p = str(tmp_path / "r.bin")
    rp.write(p)
    back = Replay.read(p)
    assert back.nb_threads == rp.nb_threads
    assert np.array_equal(back.table.keys, rp.table.keys)
    assert np.array_equal(back.table.entry_off, rp.table.entry_off)
    assert back.table.entries.tobytes() == rp.table.entries.tobytes()
    assert back.table.string_pool == rp.table.string_pool
    assert len(back.buffers) == len(rp.buffers)
    for a, b in zip(back.buffers, rp.buffers):
        assert (a.thread_rank, a.access_type, a.data_tail, a.data_head) == (b.thread_rank, b.access_type, b.data_tail, b.data_head)
        assert np.array_equal(a.ring, b.ring)


def test_generator_is_deterministic():
    a = generate(SynthConfig(nb_samples=5000, nb_intervals=100, seed=11))
    b = generate(SynthConfig(nb_samples=5000, nb_intervals=100, seed=11))
    assert a.table.entries.tobytes() == b.table.entries.tobytes()
    assert all(np.array_equal(x.ring, y.ring) for x, y in zip(a.buffers, b.buffers))


def test_copy_buffer_semantics():
    """__copy_buffer (mem_sampling.c:675-738): [tail, head) with wrap; empty
    segments are dropped."""
    ring = np.arange(100, dtype=np.uint8)
    assert np.array_equal(Buffer(0, 0, ring, 10, 30).linear(), ring[10:30])
    wrapped = Buffer(0, 0, ring, 90, 8).linear()
    assert np.array_equal(wrapped, np.concatenate([ring[90:], ring[:8]]))
    assert Buffer(0, 0, ring, 42, 42).linear().shape[0] == 0


def test_generator_shape():
    cfg = SynthConfig(nb_samples=50_000, nb_intervals=500, seed=5)
    rp = generate(cfg)
    t = rp.table
    t.validate()
    assert rp.nb_records() == cfg.nb_samples
    # every buffer fits a 128 KiB ring (mem_sampling.c:298)
    assert max(b.ring.shape[0] for b in rp.buffers) <= 3276 * RECORD_BYTES
    # address reuse -> keys with two entries; globals share one size and a NULL rip
    assert np.any(np.diff(t.entry_off.astype(np.int64)) == 2)
    glob = t.entries[t.entries["mem_type"] == 1]
    assert glob.shape[0] == cfg.nb_globals and np.all(glob["caller_rip"] == 0)
    assert t.entries[-1]["mem_type"] == 2  # [stack]
    # analysis order is newest capture first (LIFO list)
    first_ts = [int(np.frombuffer(b.ring[8:16].tobytes(), "<u8")[0]) for b in rp.buffers]
    assert first_ts[0] >= first_ts[-1]


def test_flatten_insertions_lifo():
    keys, off, order = flatten_insertions([30, 10, 30, 20, 10, 30])
    assert list(keys) == [10, 20, 30]
    assert list(off) == [0, 2, 3, 6]
    assert list(order) == [4, 1, 3, 5, 2, 0]


def test_packed_alignment():
    rp = generate(SynthConfig(nb_samples=9000, nb_intervals=50, lost_frac=5e-3, seed=2))
    arena, offs, lens, ranks, acc = rp.packed()
    assert np.all(offs % 16 == 0)
    lin = rp.linear_buffers()
    for (r, a, data), o, n in zip(lin, offs, lens):
        assert np.array_equal(arena[int(o):int(o) + int(n)], data)


def test_c_replay_writer_matches_python(tmp_path):
    """Capture bridge: a replay recorded through the C-ABI
    writer holds the same table, pools and buffers as the Python writer's, and
    the oracle's report on it is byte-identical."""
    import pyoracle
    from numamma_amd.engine import write_replay_c
    from numamma_amd.replay import Replay, SynthConfig, generate

    rp = generate(SynthConfig(nb_samples=30_000, nb_intervals=400, lost_frac=1e-3, wrap_one=True, seed=41))
    pa, pb = str(tmp_path / "py.bin"), str(tmp_path / "c.bin")
    rp.write(pa)
    write_replay_c(pb, rp)
    a, b = Replay.read(pa), Replay.read(pb)
    assert a.nb_threads == b.nb_threads
    assert np.array_equal(a.table.keys, b.table.keys) and np.array_equal(a.table.entry_off, b.table.entry_off)
    plain = [f for f in a.table.entries.dtype.names if f not in ("callstack_off", "caller_off")]
    for f in plain:
        assert np.array_equal(a.table.entries[f], b.table.entries[f]), f
    for ea, eb in zip(a.table.entries, b.table.entries):  # pools compared by content
        n = int(ea["callstack_size"])
        if ea["has_callstack"]:
            assert np.array_equal(a.table.callstack_pool[ea["callstack_off"]:ea["callstack_off"] + n],
                                  b.table.callstack_pool[eb["callstack_off"]:eb["callstack_off"] + n])
        for t, e in ((a.table, ea), (b.table, eb)):
            assert (int(e["caller_off"]) == 0xFFFFFFFF) == (int(ea["caller_off"]) == 0xFFFFFFFF)
        if int(ea["caller_off"]) != 0xFFFFFFFF:
            sa = a.table.string_pool[int(ea["caller_off"]):].split(b"\0")[0]
            sb = b.table.string_pool[int(eb["caller_off"]):].split(b"\0")[0]
            assert sa == sb
    assert len(a.buffers) == len(b.buffers)
    for x, y in zip(a.buffers, b.buffers):
        assert (x.thread_rank, x.access_type, x.data_tail, x.data_head) == (y.thread_rank, y.access_type,
                                                                           y.data_tail, y.data_head)
        assert np.array_equal(x.ring, y.ring)
    outs = []
    for p in (pa, pb):
        d = str(tmp_path / ("o_" + os.path.basename(p)))
        pyoracle.run(p, d, d + ".txt", d + "_raw.bin")
        outs.append((open(d + ".txt", "rb").read(), open(d + "_raw.bin", "rb").read(), open(d + "/call_sites.log", "rb").read()))
    assert outs[0] == outs[1]


def test_replay_context_section(tmp_path):
    """The dump-mode context (dladdr module table, /proc/<pid>/maps) travels in
    the replay's optional trailing section, written identically by the Python
    writer and the C-ABI writer (nmg_replay_set_context); readers that do not
    use it (the oracle) are unaffected."""
    import pyoracle
    from numamma_amd.engine import write_replay_c
    from numamma_amd.replay import Replay, SynthConfig, generate

    rp = generate(SynthConfig(nb_samples=5_000, nb_intervals=50, seed=43))
    rp.modules = [(0x400000, 0x480000, 0x400000, "/usr/bin/app"), (0x480000, 0x4F0000, 0x470000, "/lib/libx.so.1")]
    rp.maps_path = "/proc/4242/maps"
    rp.maps_text = "00400000-00452000 r-xp 00000000 08:02 173521 /usr/bin/app\n"
    pa, pb = str(tmp_path / "py.bin"), str(tmp_path / "c.bin")
    rp.write(pa)
    write_replay_c(pb, rp)
    ta, tb = open(pa, "rb").read(), open(pb, "rb").read()
    assert ta[ta.index(b"NMGMODS1"):] == tb[tb.index(b"NMGMODS1"):]  # (the pools may be laid out differently)
    for p in (pa, pb):
        back = Replay.read(p)
        assert back.modules == rp.modules and back.maps_path == rp.maps_path and back.maps_text == rp.maps_text
    plain = Replay.read(pa)
    plain.modules, plain.maps_path, plain.maps_text = [], None, None
    pc = str(tmp_path / "plain.bin")
    plain.write(pc)
    outs = []
    for p in (pa, pc):
        d = str(tmp_path / ("o_" + os.path.basename(p)))
        pyoracle.run(p, d, d + ".txt", d + "_raw.bin")
        outs.append((open(d + ".txt", "rb").read(), open(d + "_raw.bin", "rb").read()))
    assert outs[0] == outs[1]
