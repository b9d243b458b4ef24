"""CPU checks of the decision-emission algebra the device relies on (SURVEY.md
§8 f3; bans.h): for every IP, replaying DynamicDecisionLists.Update
(internal/decision.go:404-439) once per trip in order leaves the same entry as
one Update with the IP's highest decision taken from the first trip that
reached it — whatever entry the IP held before the batch.  Plus the fixed-zone
timestring of LogRegexBan (internal/iptables.go:189).
"""
import datetime as dt
import random

import pytest

from banjax_amd.regex_rate_limiter import DynamicDecisionLists, format_time


def per_ip_records(trips):
    """What k_ban_reduce / k_ban_out compute: ip -> (first trip with max decision, max decision)."""
    best = {}
    for t, (ip, dec, dom) in enumerate(trips):
        if ip not in best or dec > best[ip][1]:
            best[ip] = (t, dec)
    return best


@pytest.mark.parametrize("seed", range(40))
def test_one_update_per_ip_equals_per_trip_replay(seed):
    rnd = random.Random(seed)
    ips = ["10.0.0.%d" % i for i in range(rnd.randrange(1, 8))]
    pre = {ip: (rnd.randrange(1, 5), "old.com") for ip in ips if rnd.random() < 0.5}
    trips = [(rnd.choice(ips), rnd.randrange(1, 5), "d%d.com" % rnd.randrange(4)) for _ in range(rnd.randrange(1, 60))]
    expires = 123456789

    seq, once = DynamicDecisionLists(), DynamicDecisionLists()
    for lists in (seq, once):
        for ip, (d, dom) in pre.items():
            lists.update(ip, 1, d, True, dom)
    for ip, dec, dom in trips:
        seq.update(ip, expires, dec, False, dom)
    for ip, (t, dec) in sorted(per_ip_records(trips).items(), key=lambda kv: kv[1][0]):
        once.update(ip, expires, dec, False, trips[t][2])
    assert seq.expiring == once.expiring


@pytest.mark.parametrize("ns,tz", [(1700000000_123456789, 0), (1700000000_999999999, 19800), (-1, 0), (-1_500_000_000, -3600),
                                   (0, 50400), (951782400_000000000, 0), (4102444799_000000000, -43200)])
def test_format_time_fixed_zone(ns, tz):
    sec = ns // 1_000_000_000
    want = (dt.datetime(1970, 1, 1, tzinfo=dt.timezone.utc) + dt.timedelta(seconds=sec)).astimezone(
        dt.timezone(dt.timedelta(seconds=tz))).strftime("%Y-%m-%dT%H:%M:%S")
    assert format_time(ns, tz) == want


@pytest.mark.parametrize("name", ["America/New_York", "Europe/Berlin", "Australia/Lord_Howe", "Asia/Kolkata",
                                  "America/Sao_Paulo", "Pacific/Chatham", "UTC"])
def test_zone_table_matches_zoneinfo(name):
    """The transition table handed to the device (Zone, bjx_tz_transition)
    formats every sampled instant 1970-2099 as zoneinfo does."""
    import random
    import zoneinfo
    from banjax_amd import Zone
    z, tz = Zone.named(name), zoneinfo.ZoneInfo(name)
    rnd = random.Random(1)
    secs = [rnd.randrange(0, 4102444800) for _ in range(3000)]
    for a, _ in z.transitions[:200]:
        secs += [a - 1, a, a + 1]
    for s in secs:
        want = dt.datetime.fromtimestamp(s, tz).strftime("%Y-%m-%dT%H:%M:%S")
        assert format_time(s * 1_000_000_000 + 999_999_999, z) == want, (name, s)


@pytest.mark.parametrize("name", ["Europe/Berlin", "America/New_York", "Australia/Lord_Howe", "Asia/Kolkata"])
def test_zone_from_tzif_wide_range(name):
    """Zone.named reads the zone's TZif transitions (no daily sampling) and
    expands the footer rule to 2400: offsets agree with zoneinfo from 1901 to
    2380, before the first transition (Go's lookupFirstZone) and past 2100."""
    import random
    import zoneinfo
    from banjax_amd import Zone
    z, tz = Zone.named(name), zoneinfo.ZoneInfo(name)
    rnd = random.Random(4)
    secs = [rnd.randrange(-2 ** 31, 13_000_000_000) for _ in range(4000)]
    for a, _ in z.transitions:
        secs += [a - 1, a]
    for s in secs:
        assert z.offset_at(s) == int(dt.datetime.fromtimestamp(s, tz).utcoffset().total_seconds()), (name, s)
