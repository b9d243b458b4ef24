tools/gpu_session.sh "pytest_gpu|600|python -m pytest tests -m gpu -q -x -p no:cacheprovider" "bench_full|500|python bench.py --steps 3 --warmup 1 --cpu-sample 100000" "stats|200|python -c \"
import workloads as W, json
from banjax_amd import Config, Engine, Ruleset
w=W.scaled(W.CFG3, 10_000_000, n_ips=1_000_000); cfg=Config.from_yaml(w.rules_yaml); rs=Ruleset(cfg)
e=Engine(); e.set_decision_lists(cfg.decision_entries)
t,nb=w.device_lines(0)
for i in range(3): o=e.process(rs,None,w.now_ns(),device_ptr=t.data_ptr(),nbytes=nb)
print(json.dumps({'phases':e.phase_ms(),'stats':e.scan_stats(),'match_ms':o.match_kernel_ms,'lines':o.n_lines,'results':o.n_results}))
modes={}
for i in range(len(rs)): st,cl,fl=rs.rule_info(i); modes[(fl>>8)&0xff]=modes.get((fl>>8)&0xff,0)+1
print('modes',modes)
\""
