"""Generate the committed rule data and golden fixtures from the read-only reference.

Runs ONLY in the build container (where /root/reference exists); its outputs are committed, so
nothing on the GPU box reads the reference.  Outputs:

  context-based-pii_amd/rules/dlp_config.json   data: main_service/dlp_config.yaml:1-199 as JSON
                                                (the reference has no LICENSE file)
  tests/golden/transcripts.json                 data: final_transcript/ecommerce_transcript_{1,2,3}.json
  tests/golden/ref_context.json                 outputs of the reference's OWN functions:
        * extract_expected_pii (main_service/main.py:558-578) on every transcript entry and on the
          synthetic agent bank sample
        * the request call_dlp_for_redaction (main_service/main.py:580-726) sends for each
          expected_pii_type (captured from a stub dlp_client; no network)
  tests/golden/oracle_transcripts.json          the oracle's replay of the 3 transcripts (regression pin)

The two reference functions are extracted from main.py's AST and exec'd with stubbed globals
(DLP_CONFIG from the YAML, a capturing dlp_client, dlp_v2.Likelihood.VERY_LIKELY = 5); the rest of
main.py (Flask, Redis, Secret Manager) is never imported.
"""
from __future__ import annotations

import ast
import copy
import json
import logging
import os
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, REPO)


def load_reference_functions(cfg):
    src = open(os.path.join(REF, "main_service", "main.py")).read()
    tree = ast.parse(src)
    wanted = {"extract_expected_pii", "call_dlp_for_redaction"}
    mod = ast.Module(body=[n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in wanted],
                     type_ignores=[])

    class _Lik:
        VERY_LIKELY = 5

    class _DlpV2:
        Likelihood = _Lik

    class _Item:
        def __init__(self, v):
            self.value = v

    class _Resp:
        def __init__(self, v):
            self.item = _Item(v)

    class CapturingClient:
        def __init__(self):
            self.requests = []

        def deidentify_content(self, request):
            self.requests.append(copy.deepcopy(request))
            return _Resp(request["item"]["value"])

    class _E(Exception):
        pass

    client = CapturingClient()
    g = {"DLP_CONFIG": cfg, "logger": logging.getLogger("ref"), "dlp_client": client, "dlp_v2": _DlpV2,
         "GCP_PROJECT_ID_FOR_SECRETS": "test-project", "NotFound": type("NotFound", (_E,), {}),
         "PermissionDenied": type("PermissionDenied", (_E,), {}),
         "MethodNotImplemented": type("MethodNotImplemented", (_E,), {}),
         "GoogleAPICallError": type("GoogleAPICallError", (_E,), {})}
    exec(compile(mod, "main.py", "exec"), g)
    return g["extract_expected_pii"], g["call_dlp_for_redaction"], client


def main():
    with open(os.path.join(REF, "main_service", "dlp_config.yaml")) as f:
        cfg = yaml.safe_load(f)
    rules_out = os.path.join(REPO, "context-based-pii_amd", "rules", "dlp_config.json")
    with open(rules_out, "w") as f:
        json.dump({"_source": "iyngr/context-based-pii main_service/dlp_config.yaml (converted to JSON)",
                   **cfg}, f, indent=1)

    transcripts = {}
    for i in (1, 2, 3):
        with open(os.path.join(REF, "final_transcript", f"ecommerce_transcript_{i}.json")) as f:
            d = json.load(f)
        transcripts[f"ecommerce_transcript_{i}"] = {
            "conversation_id": d["conversation_info"]["conversation_id"],
            "entries": [{"i": e["original_entry_index"], "role": e["role"], "ts": e["start_timestamp_usec"],
                         "text": e["text"]} for e in d["entries"]]}
    gold = os.path.join(REPO, "tests", "golden")
    os.makedirs(gold, exist_ok=True)
    with open(os.path.join(gold, "transcripts.json"), "w") as f:
        json.dump(transcripts, f, indent=1)

    # ---- reference outputs (fresh config per call: the reference leaks state across calls) ----
    extract, _, _ = load_reference_functions(copy.deepcopy(cfg))
    ctx = {"transcripts": {}, "synthetic_agent": [], "requests": {}}
    for name, t in transcripts.items():
        ctx["transcripts"][name] = [[e["i"], e["role"], extract(e["text"])] for e in t["entries"]]
    import importlib
    synth = importlib.import_module("context-based-pii_amd.synth")
    bank = synth.agent_bank_sample(400, seed=20250718)
    for text in bank:
        ctx["synthetic_agent"].append([text, extract(text)])
    probe_types = [None] + list(cfg["context_keywords"].keys()) + ["PERSON_NAME", "PASSPORT_NUMBER_X"]
    for t in probe_types:
        _, call, client = load_reference_functions(copy.deepcopy(cfg))
        call("probe", {"expected_pii_type": t} if t else None)
        req = client.requests[-1]
        ctx["requests"][str(t)] = {k: v for k, v in req.items() if k not in ("parent", "item")}
    # the shallow-copy leak (A.7), recorded for DESIGN.md: two calls on ONE config
    _, call, client = load_reference_functions(copy.deepcopy(cfg))
    call("probe", {"expected_pii_type": "PERSON_NAME"})
    call("probe", None)
    call("probe", {"expected_pii_type": "CREDIT_CARD_NUMBER"})
    ctx["leak_probe"] = {"info_types_after": len(client.requests[-1]["inspect_config"]["info_types"]),
                         "rule_sets_after": len(client.requests[-1]["inspect_config"]["rule_set"])}
    with open(os.path.join(gold, "ref_context.json"), "w") as f:
        json.dump(ctx, f, indent=1)

    # ---- oracle replay of the three transcripts (regression pin for the oracle itself) ----------
    from oracle import pii_oracle as O
    rc = O.RuleConfig.load()
    rep = {}
    for name, t in transcripts.items():
        rows = [(t["conversation_id"], O.ROLE_AGENT if e["role"] == "AGENT" else O.ROLE_CUSTOMER,
                 e["text"].encode(), e["ts"]) for e in t["entries"]]
        res = O.process_rows(rows, rc)
        rep[name] = [{"i": e["i"], "redacted": r[0].decode(), "context_used": r[2], "context_stored": r[3],
                      "spans": [[f.start, f.end, rc.type_names[f.type_id], f.likelihood] for f in r[1]]}
                     for e, r in zip(t["entries"], res)]
    with open(os.path.join(gold, "oracle_transcripts.json"), "w") as f:
        json.dump(rep, f, indent=1)
    print("fixtures written")


if __name__ == "__main__":
    main()
