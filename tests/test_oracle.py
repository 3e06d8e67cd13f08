"""The CPU oracle pinned against the reference's own outputs (tests/golden/ref_context.json, produced
by running main_service/main.py's extract_expected_pii / call_dlp_for_redaction, see
oracle/gen_fixtures.py) and against the SURVEY Appendix B known answers."""
import copy
import json
import os

import pytest

from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(GOLD, "ref_context.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def transcripts():
    with open(os.path.join(GOLD, "transcripts.json")) as f:
        return json.load(f)


def test_extract_expected_pii_matches_reference_on_transcripts(ref, transcripts, oracle_cfg):
    from oracle import pii_oracle as O
    for name, t in transcripts.items():
        got = [[e["i"], e["role"], O.extract_expected_pii(e["text"], oracle_cfg)] for e in t["entries"]]
        assert got == ref["transcripts"][name]


def test_extract_expected_pii_matches_reference_on_synthetic(ref, oracle_cfg):
    from oracle import pii_oracle as O
    assert len(ref["synthetic_agent"]) == 400
    for text, exp in ref["synthetic_agent"]:
        assert O.extract_expected_pii(text, oracle_cfg) == exp, text


def test_appendix_b1_quirks(oracle_cfg):
    from oracle import pii_oracle as O
    assert O.extract_expected_pii("is now being processed", oracle_cfg) == "US_EMPLOYER_IDENTIFICATION_NUMBER"
    assert O.extract_expected_pii("your US Driver's License number?", oracle_cfg) == "STREET_ADDRESS"
    assert O.extract_expected_pii("The IP address associated", oracle_cfg) == "STREET_ADDRESS"
    assert O.extract_expected_pii("a Border Crossing Card number?", oracle_cfg) == "CREDIT_CARD_NUMBER"
    assert O.extract_expected_pii("Hello there", oracle_cfg) is None


def _canon(insp):
    """Order-preserving canonical form of an inspect_config (likelihood enums as ints)."""
    d = copy.deepcopy(insp)
    for rs in d.get("rule_set", []):
        for r in rs.get("rules", []):
            adj = r.get("hotword_rule", {}).get("likelihood_adjustment")
            if adj and "fixed_likelihood" in adj and isinstance(adj["fixed_likelihood"], str):
                from oracle.pii_oracle import LIKELIHOOD
                adj["fixed_likelihood"] = LIKELIHOOD[adj["fixed_likelihood"]]
    return json.dumps(d, sort_keys=True)


def test_context_merge_matches_reference_requests(ref, oracle_cfg):
    """a6: the request the reference sends for every expected_pii_type (main.py:609-726)."""
    for t, req in ref["requests"].items():
        et = None if t == "None" else t
        insp, dynamic = oracle_cfg.merged_inspect_config(et)
        if et is None:
            assert "inspect_template_name" in req and "inspect_config" not in req and not dynamic
            # template == YAML inspect_config (deployment/update_dlp_templates.py:49-51)
            assert _canon(insp) == _canon(oracle_cfg.raw["inspect_config"])
        else:
            assert dynamic and "inspect_config" in req and "inspect_template_name" not in req
            assert _canon(insp) == _canon(req["inspect_config"]), t
        assert "deidentify_template_name" in req and "deidentify_config" not in req


def test_compiler_context_merge_equals_oracle(ref, compiled, oracle_cfg):
    for t in ref["requests"]:
        et = None if t == "None" else t
        a = compiled.rules.merged_inspect_config(et)
        b, _ = oracle_cfg.merged_inspect_config(et)
        assert _canon(a) == _canon(b)


def test_leak_is_not_reproduced(ref, oracle_cfg):
    # the reference leaks the PERSON_NAME rule set into later requests (A.7); the restatement is stateless
    assert ref["leak_probe"] == {"info_types_after": 20, "rule_sets_after": 6}
    oracle_cfg.merged_inspect_config("PERSON_NAME")
    insp, _ = oracle_cfg.merged_inspect_config("CREDIT_CARD_NUMBER")
    assert len(insp["info_types"]) == 19 and len(insp["rule_set"]) == 5


def test_checksums_b4():
    from oracle import pii_oracle as O
    assert O.v_luhn(b"4141-1212-2323-5009") and O.v_luhn(b"490154203237518")
    for s in (b"9876543210", b"12345", b"987654321", b"8675309"):
        assert not O.v_luhn(s)
    assert O.v_iban(b"DE89370400440532013000") and not O.v_iban(b"DE89370400440532013001")
    assert O.v_swift(b"COBADEFFXXX") and not O.v_swift(b"COBAQQFFXXX")
    assert O.v_ssn(b"123-45-6789") and not O.v_ssn(b"666-45-6789") and not O.v_ssn(b"912-45-6789")
    assert O.v_ein(b"12-1234567") and not O.v_ein(b"07-1234567")
    assert O.v_ipv4(b"198.51.100.10") and not O.v_ipv4(b"198.51.100.256")
    assert O.v_nanp(b"555-555-5555") and not O.v_nanp(b"155-555-5555")


def test_appendix_b3_custom_regex_hits(transcripts, oracle_cfg):
    from oracle import pii_oracle as O
    t1 = {e["i"]: e["text"].encode() for e in transcripts["ecommerce_transcript_1"]["entries"]}
    t2 = {e["i"]: e["text"].encode() for e in transcripts["ecommerce_transcript_2"]["entries"]}
    handle = next(d for d in oracle_cfg.detectors if d.type_name == "SOCIAL_HANDLE")
    assert [m.span() for m in handle.regex.finditer(t1[15])] == [(112, 122)]
    assert [m.span() for m in handle.regex.finditer(t1[16])] == [(18, 30)]
    assert [m.span() for m in handle.regex.finditer(t1[7])] == [(25, 37)]
    alien = next(d for d in oracle_cfg.detectors if d.type_name == "ALIEN_REGISTRATION_NUMBER")
    assert [m.span() for m in alien.regex.finditer(t2[24])] == [(20, 30)]
    bcc = next(d for d in oracle_cfg.detectors if d.type_name == "BORDER_CROSSING_CARD")
    assert [m.span() for m in bcc.regex.finditer(t2[26])] == [(10, 18)]
    # A.5: the handle inside the e-mail is excluded
    red, fs = O.redact(t1[7], oracle_cfg)
    assert red == b"Yes, my email is [EMAIL_ADDRESS]." and len(fs) == 1


def test_oracle_transcripts_regression(transcripts, oracle_cfg):
    from oracle import pii_oracle as O
    with open(os.path.join(GOLD, "oracle_transcripts.json")) as f:
        gold = json.load(f)
    for name, t in transcripts.items():
        rows = [(name, O.ROLE_AGENT if e["role"] == "AGENT" else O.ROLE_CUSTOMER, e["text"].encode(), e["ts"])
                for e in t["entries"]]
        for g, (red, fs, used, stored) in zip(gold[name], O.process_rows(rows, oracle_cfg)):
            assert red.decode() == g["redacted"]
            assert [[f.start, f.end, oracle_cfg.type_names[f.type_id], f.likelihood] for f in fs] == g["spans"]
            assert used == g["context_used"] and stored == g["context_stored"]


def test_ttl_semantics():
    from oracle import pii_oracle as O
    st = O.ContextStore(90)
    st.set("c", "CVV_NUMBER", b"x", 0)
    assert st.get("c", 89_999_999)[0] == "CVV_NUMBER"
    assert st.get("c", 90_000_000) is None


def test_realtime_join_and_window(oracle_cfg):
    from oracle import pii_oracle as O
    agent = b"Can you confirm the CVV on your card?"
    # 'cvv' hotword sits in the agent line, within 50 B of the customer's digits
    assert O.realtime_redact(agent, b"123", oracle_cfg, "CREDIT_CARD_NUMBER") == b"[CVV_NUMBER]"
    assert O.realtime_redact(None, b"123", oracle_cfg, None) == b"123"
    w = O.window_rescan([b"my cvv", b"is 123"], oracle_cfg, None)
    assert w == b"my cvv\nis [CVV_NUMBER]"
