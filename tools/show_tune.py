import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["summary"].items():
    print(f"{k:24s} wall_min={v['wall_ms_min']:9.2f} ms  proj={v['proj_us_min']:8.2f} us  resid={v['resid']:.6e}  {v['breakdown_ms']}")
