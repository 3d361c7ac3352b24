import json, os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from benchmarks.sections import protocol_sizes
r = protocol_sizes(torch.device("cuda", 0), cases=((262144, torch.bfloat16, 0, 3000), (1 << 20, torch.bfloat16, 0, 3000),
                                                   (4 << 20, torch.bfloat16, 0, 2000)))
print(json.dumps({"cfg": sys.argv[1], **{k: {f: v.get(f) for f in ("us_per_round", "round_interval_p50_us", "validated", "error")}
                                          for k, v in r.items() if isinstance(v, dict)}}), flush=True)
