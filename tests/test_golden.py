"""Golden consumeLine vectors (tests/golden/*.json.gz, made by
tests/golden/make_golden.py): the oracle must reproduce them on the CPU, and
the HIP engine behind the C ABI must reproduce them bit for bit on the GPU."""
import base64
import glob
import gzip
import json
import os

import pytest

from banjax_amd import Config, Engine, MockBanner, RegexRateLimiter
from oracle import oracle as O
from tests.parity import oracle_config

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json.gz")))
NAMES = [os.path.basename(p)[:-len(".json.gz")] for p in GOLDEN]


def load(path):
    with gzip.open(path, "rt", encoding="utf-8") as f:
        return json.load(f)


def test_golden_set_present():
    assert {"consume_line_sequence", "fixture_config", "edge_lines", "tile_geometry", "workload_cfg1",
            "workload_cfg2", "workload_cfg3", "workload_cfg4", "workload_cfg5", "integration_challengeme",
            "integration_rates"} <= set(NAMES)


@pytest.mark.parametrize("path", GOLDEN, ids=NAMES)
def test_oracle_reproduces_golden(path):
    fx = load(path)
    cfg = Config.from_yaml(fx["config_yaml"])
    oc = oracle_config(cfg)
    st = O.State()
    n_rules = len(cfg.all_rules())
    for b in fx["batches"]:
        if "sighup_yaml" in b:  # banjax.go:101-115: Reload, then DynamicDecisionLists.Clear
            cfg = Config.from_yaml(b["sighup_yaml"])
            oc = oracle_config(cfg)
            n_rules = len(cfg.all_rules())
            st.decisions_clear()
        data = base64.b64decode(b["log_b64"])
        flags, res, consumed = st.consume(oc, data, b["now_ns"], cap=(data.count(b"\n") + 1) * (n_rules + 1))
        assert consumed == b["consumed"]
        assert flags == b["flags"]
        assert [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded]
                for r in res] == b["results"]
    assert len(st) == fx["state_len"]
    for ip, nm, hits, start in fx["states"]:
        g = st.get(base64.b64decode(ip), nm)
        assert (g is None and hits is None) or g == (hits, start)
    assert st.decisions_len() == fx["decisions_len"]
    assert [l for l in st.ban_log().split("\n") if l] == fx["ban_log"]


@pytest.fixture(scope="module")
def engine():
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("device_bans", [False, True], ids=["host_banner", "device_bans"])
@pytest.mark.parametrize("path", GOLDEN, ids=NAMES)
def test_engine_reproduces_golden(engine, path, device_bans):
    """device_bans: the decisions and ban-log lines come from the GPU emission
    (bjx_batch_bans) instead of the host Banner replay of the trip list."""
    fx = load(path)
    cfg = Config.from_yaml(fx["config_yaml"])
    engine.state_clear()
    lim = RegexRateLimiter(cfg, engine=engine, banner=MockBanner(), device_bans=device_bans)
    for b in fx["batches"]:
        if "sighup_yaml" in b:
            lim.sighup(Config.from_yaml(b["sighup_yaml"]))
        data = base64.b64decode(b["log_b64"])
        _, out = lim.consume_lines(data, b["now_ns"], want_results=True)
        assert out.consumed_bytes == b["consumed"]
        assert list(out.line_flags) == b["flags"]
        got = [[r.line_idx, r.rule_idx, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded]
               for r in out.results]
        assert got == b["results"]
        assert [[t.line_idx, t.rule_idx] for t in out.trips] == b["trips"]
    assert engine.state_len() == fx["state_len"]
    for ip, nm, hits, start in fx["states"]:
        g = engine.state_get(base64.b64decode(ip), nm)
        assert (g is None and hits is None) or g == (hits, start), (ip, nm, g, hits, start)
    dl = lim.banner.decision_lists.expiring
    assert len(dl) == fx["decisions_len"]
    for ip, dec, exp, dom in fx["decisions"]:
        d = dl[base64.b64decode(ip).decode("utf-8", "surrogateescape")]
        assert (d.decision, d.expires_ns, d.domain) == (dec, exp, dom)
    # oracle ban log lines: "0 <json>" (Banner.Logger) / "1 <json>" (LoggerTemp, disable_logging hosts)
    glog = ["0 " + l for l in lim.banner.ban_log] + ["1 " + l for l in lim.banner.ban_log_temp]
    if lim.banner.ban_log_temp:
        assert sorted(glog) == sorted(fx["ban_log"])
    else:
        assert glog == fx["ban_log"]
    if fx["banned_ip"]:
        assert lim.banner.banned_ip == fx["banned_ip"]
