#!/usr/bin/env python3
"""One line from a tools/ab.py JSON (its stdout may carry a runtime warning first):
median ms per variant, "(DIFF)" where a variant's output differs from the first's."""
import json
import sys

t = open(sys.argv[1]).read()
d = json.loads(t[t.index("{"):])
print(" ".join(f"{k}:{v['median_ms']}" + ("" if v["bitexact_vs_first"] else "(DIFF)") for k, v in d["variants"].items()),
      "steps", d["steps"])
