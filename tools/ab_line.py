"""One A/B row from a bench.py JSON line on stdin: variant, img/s, ms/step, class ms per step."""
import json
import sys

d = json.loads(sys.stdin.read())
ms = {k.split()[0] + ("" if "(" not in k else ":" + k.split("(")[1].split()[0]): v["ms"] for k, v in d["roofline"]["classes"].items()}
print(sys.argv[1], d["value"], d["ms_per_step"], " ".join(f"{k}={m}" for k, m in ms.items()))
