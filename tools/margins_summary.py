"""Summarise a parity-margins file (tests/conftest.py check(): one JSON line per GPU test with every tolerance check's
achieved error and bound) as a markdown table, or only the rows matching substrings:

  python tools/margins_summary.py profiles/r06/parity_margins.jsonl [substr ...]
"""
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
keys = [k for k in sys.argv[2:] if k != "--stats"]
if "--stats" in sys.argv[2:]:
    import statistics

    m = [c["bound"] / c["achieved"] for r in rows for c in r["checks"]
         if c["bound"] is not None and c["op"] != "==" and c["achieved"] > 0]
    z = sum(1 for r in rows for c in r["checks"] if c["bound"] is not None and c["op"] != "==" and c["achieved"] == 0)
    b = sum(1 for r in rows for c in r["checks"] if c["op"] == "==")
    print(f"{len(m)} bounded tolerance checks (+{z} at exactly 0, {b} bitwise): bound / achieved median "
          f"{statistics.median(m):.1f}, min {min(m):.2f}; < 3x: {sum(x < 3 for x in m)}, < 10x: {sum(x < 10 for x in m)}, "
          f"> 1000x: {sum(x > 1000 for x in m)}")
    sys.exit(0)
n_chk = sum(len(r["checks"]) for r in rows)
print(f"{len(rows)} tests ({sum(r['outcome'] == 'passed' for r in rows)} passed), {n_chk} recorded quantities, "
      f"lib {rows[0].get('lib_sha16', '')} head {rows[0].get('head', '')}\n")
print("| test | quantity | achieved | bound | bound / achieved |")
print("|---|---|---|---|---|")
for r in rows:
    t = r["test"].split("::")[-1].replace("|", "\\|")
    for c in r["checks"]:
        c = dict(c, name=c["name"].replace("|", "\\|"))
        if keys and not any(k in t or k in c["name"] for k in keys):
            continue
        b = c["bound"]
        if b is None:
            print(f"| {t} | {c['name']} | {c['achieved']:.2e} | (recorded) | |")
        elif c["op"] == "==":
            print(f"| {t} | {c['name']} | {c['achieved']:.3g} | == {b:g} | bitwise |")
        else:
            m = b / c["achieved"] if c["achieved"] > 0 else float("inf")
            print(f"| {t} | {c['name']} | {c['achieved']:.2e} | {c['op']} {b:.2e} | {m:.1f} |")
