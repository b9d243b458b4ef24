import json,sys
for f in sys.argv[1:]:
    try:
        d=json.loads(open(f).read().strip().splitlines()[-1])
        print(f, "value %.4g" % d["value"], "ms", d["ms_per_step"], d["config"]["phase_ms_last_step_rank0"], "jobs", d["config"]["scan_stats_last_step_rank0"]["dfa_jobs"])
    except Exception as e:
        print(f, "ERR", e)
