"""bjx_node_*: several engines behind one handle, the exchange inside the library.

The engines share GPU 0 here (the box has one GPU; the library takes the
same-device copy path instead of its RCCL clique, which needs one GPU per
engine); the RCCL path itself runs with one engine forced through the exchange.  Every batch is checked
bit-exact against one oracle over the whole stream: per-line flags, the
RuleResults and trips in reference order, the merged decision records and
ban-log lines, and the RegexRateLimitStates spread over the shards.
"""
import pytest

import workloads as W
from banjax_amd import Config, Node
from banjax_amd.regex_rate_limiter import DynamicDecisionLists
from oracle import oracle as O
from tests.parity import oracle_config

pytestmark = pytest.mark.gpu


def _check_batch(cfg, st, oc, data, now_ns, out, bans, dl, blog, copy=True):
    oflags, ores, _ = st.consume(oc, data, now_ns, cap=(data.count(b"\n") + 1) * (len(cfg.all_rules()) + 1))
    exp = [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded] for r in ores]
    assert out.n_lines == data.count(b"\n")
    if copy:
        assert list(out.line_flags) == oflags
        got = [[x.line_idx, x.rule_idx, x.rule_pos, x.skip_host, x.seen_ip, x.match_type, x.exceeded] for x in out.results]
        assert got == exp
    trips = out.trips
    assert [(t.line_idx, t.rule_idx) for t in trips] == [(r[0], r[1]) for r in exp if r[6]]
    for t in trips[:50]:  # offsets are relative to the whole batch
        line = data[t.line_offset:t.line_offset + t.line_len]
        assert data[t.line_offset + t.line_len:t.line_offset + t.line_len + 1] == b"\n"
        assert line.split(b" ")[1] == line[t.ip_off:t.ip_off + t.ip_len]
    # merged decision records: replay as the Banner does, in trip order
    assert bans.n_trips == len(trips)
    prev = -1
    for r, rec in enumerate(bans.ips):
        t = trips[int(rec["trip_idx"])]
        assert int(rec["trip_idx"]) > prev
        prev = int(rec["trip_idx"])
        line = data[t.line_offset:t.line_offset + t.line_len]
        assert bans.ip(r) == line[t.ip_off:t.ip_off + t.ip_len]
        host = line[t.host_off:t.host_off + t.host_len]
        dl.update(bans.ip(r).decode(), int(rec["expires_ns"]), int(rec["decision"]), False, host.decode())
    blog += ["%d %s" % (kind - 1, line.decode()) for kind, line in bans.lines()]
    return len(trips)


@pytest.mark.parametrize("wl,n_engines,device_input,rccl,copy", [
    (("cfg3", 2000), 2, False, False, True),
    (("cfg5", 3000), 3, True, False, True),
    (("cfg1", 500), 4, False, False, True),
    (("cfg3", 2000), 1, True, False, True),
    (("cfg5", 3000), 1, True, True, True),
    (("cfg3", 2000), 1, False, True, True),
    (("cfg3", 2000), 2, False, False, False),
    (("cfg5", 3000), 3, True, False, False),
    (("cfg3", 2000), 1, False, True, False),
])
def test_node_matches_one_oracle(wl, n_engines, device_input, rccl, copy, monkeypatch):
    """rccl: one engine whose batches still go through the library's exchange
    (BJX_NODE_FORCE_EXCHANGE), moved by the RCCL path (a one-GPU clique from
    ncclCommInitAll, ncclSend / ncclRecv to itself) that a node of distinct
    GPUs uses between all of them.  copy=False: trips-only batches, whose
    owners send back trip lists (bjx_apply_events_trips /
    bjx_finish_batch_trips) instead of per-event outcomes."""
    import torch

    steps, per = 3, 12_000
    w = W.scaled(W.ALL[wl[0]], steps * per, n_ips=wl[1])
    cfg = Config.from_yaml(w.rules_yaml)
    from banjax_amd import Ruleset
    rs = Ruleset(cfg)
    if rccl:
        monkeypatch.setenv("BJX_NODE_FORCE_EXCHANGE", "1")
        monkeypatch.setenv("BJX_NODE_EXCHANGE", "rccl")
    node = Node([0] * n_engines)
    assert len(node) == n_engines
    assert node.exchange == ("rccl" if rccl else "copies")
    node.set_decision_lists(cfg.decision_entries)
    node.set_ban_options(cfg.expiring_decision_ttl_seconds)
    oc = oracle_config(cfg)
    st = O.State()
    dl, blog, n_trips = DynamicDecisionLists(), [], 0
    keep = []
    for s in range(steps):
        data = w.host_lines(s * per, per)
        now = w.now_ns(s * per, per)
        if device_input:
            # uneven chunks on line boundaries, each copied to "its" GPU
            lines = data.split(b"\n")[:-1]
            cuts = [0] + sorted({(len(lines) * (k + 1)) // (n_engines + 1) for k in range(n_engines - 1)}) + [len(lines)]
            chunks = []
            for a, b in zip(cuts, cuts[1:]):
                blob = b"".join(ln + b"\n" for ln in lines[a:b])
                t = torch.frombuffer(bytearray(blob or b"\0"), dtype=torch.uint8).to("cuda:0")
                keep.append(t)
                chunks.append((t.data_ptr(), len(blob)))
            out = node.process_chunks(rs, chunks, now, copy_results=copy, emit_bans=True)
        else:
            out = node.process(rs, data, now, copy_results=copy, emit_bans=True)
        assert out.consumed_bytes == len(data)
        n_trips += _check_batch(cfg, st, oc, data, now, out, node.bans(), dl, blog, copy)
    assert n_trips > 0
    assert len(dl.expiring) == st.decisions_len()
    for ip, d in dl.expiring.items():
        assert tuple(st.decision(ip)[:3]) == (d.decision, d.expires_ns, d.domain), ip
    assert blog == [ln for ln in st.ban_log().split("\n") if ln]
    # RegexRateLimitStates over the shards: Len, Get, String, occupancy
    assert node.state_len() == len(st)
    names = sorted(set(r.rule for r in cfg.all_rules()))
    first = w.host_lines(0, per).split(b"\n")
    for ln in first[:60]:
        ip = ln.split(b" ")[1]
        for nm in names:
            assert node.state_get(ip, nm) == st.get(ip, nm), (ip, nm)
    dump = node.state_dump()
    assert sum(1 for ln in dump.split("\n") if ln and not ln.startswith("\t")) == len(st)
    stats = node.state_stats()
    assert stats["ips"] == len(st) and stats["states"] >= len(st)
    node.state_clear()
    assert node.state_len() == 0
    node.close()


def test_node_rejects_chunk_without_newline():
    import torch

    from banjax_amd import Ruleset
    from banjax_amd._lib import BanjaxGpuError
    w = W.scaled(W.CFG3, 1000, n_ips=100)
    cfg = Config.from_yaml(w.rules_yaml)
    rs = Ruleset(cfg)
    node = Node([0, 0])
    data = w.host_lines(0, 1000)
    cut = data.index(b"\n", len(data) // 2) - 3  # mid-line
    a = torch.frombuffer(bytearray(data[:cut]), dtype=torch.uint8).to("cuda:0")
    b = torch.frombuffer(bytearray(data[cut:]), dtype=torch.uint8).to("cuda:0")
    with pytest.raises(BanjaxGpuError):
        node.process_chunks(rs, [(a.data_ptr(), cut), (b.data_ptr(), len(data) - cut)], w.now_ns(0, 1000))
    # a host batch splits itself on line boundaries, a partial tail is carried
    out = node.process(rs, data + b"1700000000.000 1.2.3.4 GET", w.now_ns(0, 1000))
    assert out.consumed_bytes == len(data) and out.n_lines == 1000
    node.close()


def test_node_rejects_oversized_ip_field():
    """bjx_event_line carries the IP length in 16 bits: a batch with an event
    line whose IP field is 64 KiB or longer fails with BJX_ERR_CAPACITY rather
    than keying the owner's state by a truncated IP.  A single engine (no
    exchange) keys it by every byte, as the oracle does."""
    from banjax_amd import Engine, Ruleset
    from banjax_amd._lib import BanjaxGpuError
    from tests.parity import Pair
    yml = """
regexes_with_rates:
  - rule: "all"
    regex: ".*"
    interval: 5
    hits_per_interval: 1
    decision: nginx_block
"""
    cfg = Config.from_yaml(yml)
    rs = Ruleset(cfg)
    big = b"1" * 70_000
    data = b"1700000000.000 1.2.3.4 GET a.com GET / HTTP/1.1\n1700000000.000 " + big + b" GET a.com GET / HTTP/1.1\n"
    node = Node([0, 0])
    with pytest.raises(BanjaxGpuError) as ei:
        node.process(rs, data, 1700000000 * 10**9)
    assert ei.value.code == -6 and "65535" in str(ei.value)
    node.close()
    eng = Engine(0)
    pair = Pair(yml, eng)
    pair.feed(data + data, 1700000000 * 10**9)
    pair.compare_state(["1.2.3.4", big.decode()])
    eng.close()


def test_node_compact_trips_match_full():
    """A node's BJX_TRIPS_COMPACT words (line offsets rebased to the whole
    batch) equal its full trip records, over three engines."""
    from banjax_amd import Ruleset

    w = W.scaled(W.CFG5, 30_000, n_ips=3_000)
    rs = Ruleset(Config.from_yaml(w.rules_yaml))
    data = w.host_lines(0, 30_000)
    now = w.now_ns(0, 30_000)
    node = Node([0] * 3)
    full = node.process(rs, data, now)
    want = [(t.line_offset, t.rule_idx) for t in full.trips]
    node.state_clear()
    import torch
    lines = data.split(b"\n")[:-1]
    cuts = [0, len(lines) // 3, 2 * len(lines) // 3, len(lines)]
    chunks, keep = [], []
    for a, b in zip(cuts, cuts[1:]):
        blob = b"".join(ln + b"\n" for ln in lines[a:b])
        t = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to("cuda:0")
        keep.append(t)
        chunks.append((t.data_ptr(), len(blob)))
    full2 = node.process_chunks(rs, chunks, now)
    want2 = [(t.line_offset, t.rule_idx) for t in full2.trips]
    node.state_clear()
    comp = node.process_chunks(rs, chunks, now, compact_trips=True)
    got = [(int(x) >> 24, int(x) & 0xFFFFFF) for x in comp.trips_compact()]
    node.close()
    assert comp.n_trips == len(want2) > 100
    assert got == want2 and want2 == want
