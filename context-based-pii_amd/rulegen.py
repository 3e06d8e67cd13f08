"""Config 5 (BASELINE.json configs[4]): a seeded rule set of 500+ custom regex and dictionary
infoTypes on top of the shipped dlp_config, and text that exercises it.

The reference has no such rule set ("Dictionaries first appear in BASELINE config 5,
which is synthetic"); its loader takes custom infoTypes, rule sets and context keywords from the same
dlp_config structure (main_service/main.py:58-66 load_dlp_config, :609-686 the context merge), so
the generated config is that structure: the shipped one + ``n_regex`` regex types + ``n_dict``
dictionary types (word lists, matched case-insensitively on word boundaries), hotword rule sets over
some of them (fixed and relative likelihood adjustments, window_before and window_after), and context
keywords for some of them (extract_expected_pii then names a custom type; the merge appends its
definition, main.py:624-634).  Everything is derived from ``seed``.
"""
from __future__ import annotations

import copy
import json
import os
import random
import re
from typing import Dict, List, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
BASE_CONFIG = os.path.join(HERE, "rules", "dlp_config.json")

_CONS = "bcdfghjklmnprstvwxz"
_VOW = "aeiou"
_LIKS = ["VERY_LIKELY", "LIKELY", "POSSIBLE", "UNLIKELY", "VERY_LIKELY", "LIKELY"]


def _word(r: random.Random, syl: int) -> str:
    return "".join(r.choice(_CONS) + r.choice(_VOW) + (r.choice(_CONS) if r.random() < 0.4 else "")
                   for _ in range(syl))


def _unique(r: random.Random, used: set, make) -> str:
    while True:
        w = make()
        if w not in used:
            used.add(w)
            return w


class Config5:
    """The generated dlp_config (``cfg``) plus what the text generator needs per custom type."""

    def __init__(self, n_regex: int = 320, n_dict: int = 200, seed: int = 5, base_path: str = BASE_CONFIG):
        r = random.Random(seed)
        with open(base_path) as f:
            base = json.load(f)
        cfg = copy.deepcopy(base)
        cfg["_source"] = f"rulegen.Config5(n_regex={n_regex}, n_dict={n_dict}, seed={seed}) over {os.path.basename(base_path)}"
        insp = cfg["inspect_config"]
        used_pfx, used_words = set(), set()
        self.samplers: Dict[str, Tuple[str, object]] = {}
        customs = []
        for i in range(n_regex):
            name = f"CUSTOM_ID_{i:03d}"
            k = i % 5
            pfx = _unique(r, used_pfx, lambda: "".join(r.choice("ABCDEFGHJKLMNPQRSTUVWXYZ") for _ in range(r.randint(2, 4))))
            n = r.randint(4, 9)
            if k == 0:
                pat, spec = rf"\b{pfx}-\d{{{n}}}\b", ("dash", pfx, n)
            elif k == 1:
                pat, spec = rf"\b{pfx}\d{{{n}}}[A-Z]\b", ("tail", pfx, n)
            elif k == 2:
                lp = pfx.lower()
                a = r.randint(3, 5)
                b = a + r.randint(1, 4)
                pat, spec = rf"\b{lp}_[a-z0-9]{{{a},{b}}}\b", ("under", lp, (a, b))
            elif k == 3:
                pat, spec = rf"\b{pfx}/\d{{2}}-\d{{{n}}}\b", ("slash", pfx, n)
            else:
                w = _unique(r, used_words, lambda: _word(r, 2))
                pat, spec = rf"(?i)\b{w}#\d{{{n}}}\b", ("hash", w, n)
            customs.append({"info_type": {"name": name}, "regex": {"pattern": pat},
                            "likelihood": r.choice(_LIKS)})
            self.samplers[name] = spec
        for i in range(n_dict):
            name = f"CUSTOM_DICT_{i:03d}"
            words = []
            for _ in range(r.randint(4, 24)):
                if r.random() < 0.2:
                    words.append(_unique(r, used_words, lambda: _word(r, r.randint(2, 3)) + " " + _word(r, 2)))
                else:
                    words.append(_unique(r, used_words, lambda: _word(r, r.randint(2, 4))))
            customs.append({"info_type": {"name": name}, "dictionary": {"word_list": {"words": words}},
                            "likelihood": r.choice(_LIKS)})
            self.samplers[name] = ("dict", words, None)
        insp["custom_info_types"] = list(insp.get("custom_info_types", [])) + customs
        names = [c["info_type"]["name"] for c in customs]
        # hotword rule sets over groups of custom types
        self.hotwords: Dict[str, List[str]] = {}
        rule_sets = []
        pool = names[:]
        r.shuffle(pool)
        for g in range(24):
            members = pool[g * 6:(g + 1) * 6]
            hws = [_unique(r, used_words, lambda: _word(r, 2)) for _ in range(r.randint(1, 3))]
            prox = {"window_before": r.choice([20, 30, 50, 60])}
            if r.random() < 0.4:
                prox["window_after"] = r.choice([10, 20, 40])
            adj = ({"fixed_likelihood": "VERY_LIKELY"} if r.random() < 0.5 else
                   {"relative_likelihood": r.choice([1, 2, -1])})
            rule_sets.append({"info_types": [{"name": n} for n in members],
                              "rules": [{"hotword_rule": {"hotword_regex": {"pattern": "(?i)(" + "|".join(hws) + ")"},
                                                          "proximity": prox, "likelihood_adjustment": adj}}]})
            for n in members:
                self.hotwords[n] = hws
        insp["rule_set"] = list(insp.get("rule_set", [])) + rule_sets
        # context keywords for some custom types (after the built-ins': first type with a hit wins)
        self.context_types = []
        ck = cfg.setdefault("context_keywords", {})
        for n in pool[24 * 6:24 * 6 + 20]:
            kw = [_unique(r, used_words, lambda: "your " + _word(r, 2))]
            ck[n] = kw
            self.context_types.append(n)
        self.cfg = cfg
        self.custom_names = names

    # ------------------------------------------------------------------ text
    def value(self, r: random.Random, name: str) -> str:
        kind, a, b = self.samplers[name]
        digits = lambda n: "".join(r.choice("0123456789") for _ in range(n))  # noqa: E731
        if kind == "dash":
            return f"{a}-{digits(b)}"
        if kind == "tail":
            return f"{a}{digits(b)}{r.choice('ABCDEFGHJKLMNPQRSTUVWXYZ')}"
        if kind == "under":
            return f"{a}_" + "".join(r.choice("abcdefghijklmnopqrstuvwxyz0123456789") for _ in range(r.randint(*b)))
        if kind == "slash":
            return f"{a}/{digits(2)}-{digits(b)}"
        if kind == "hash":
            w = a.upper() if r.random() < 0.3 else a
            return f"{w}#{digits(b)}"
        w = r.choice(a)
        return w.upper() if r.random() < 0.2 else (w.capitalize() if r.random() < 0.3 else w)

    def near_miss(self, r: random.Random, name: str) -> str:
        """a value of the type, mutated so that it may or may not still match"""
        v = self.value(r, name)
        k = r.randrange(len(v))
        return v[:k] + r.choice("0123456789-_ #xZ") + v[k + 1:]

    def utterance(self, r: random.Random, builtin_value=None) -> str:
        """filler with 0-3 custom values (sometimes after one of their hotwords, sometimes mutated)
        and now and then a built-in PII value"""
        parts = []
        for _ in range(r.randint(0, 3)):
            n = r.choice(self.custom_names)
            v = self.near_miss(r, n) if r.random() < 0.2 else self.value(r, n)
            if n in self.hotwords and r.random() < 0.4:
                hw = r.choice(self.hotwords[n])
                v = f"{hw} is {v}" if r.random() < 0.7 else f"{v} was my {hw}"
            parts.append(v)
        if builtin_value is not None and r.random() < 0.3:
            parts.append(builtin_value(r))
        fill = ["ok", "so", "the number is", "thanks", "and", "please note", "my code", "um", "right"]
        out = []
        for p in parts:
            out.append(r.choice(fill))
            out.append(p)
        out.append(r.choice(fill))
        return " ".join(out)

    def agent_utterance(self, r: random.Random) -> str:
        if self.context_types and r.random() < 0.5:
            t = r.choice(self.context_types)
            return f"Could you confirm {self.cfg['context_keywords'][t][0]} please?"
        return r.choice(["How can I help?", "One moment please.", "Thanks for waiting."])

    def build_bank(self, n_agent: int = 4096, n_customer: int = 12288, seed: int = 7):
        """an utterance bank (synth.Bank) of config-5 text: customer rows with custom (and some
        built-in) values, agent rows that name custom contexts or the built-ins' keywords"""
        from . import synth
        r = random.Random(seed)
        kws = synth._keywords()
        texts = [(self.agent_utterance(r) if r.random() < 0.5 else synth.agent_utterance(r, kws)).encode()
                 for _ in range(n_agent)]
        bv = lambda rr: synth.pii_value(rr, rr.choice(synth.PII_TYPES), rr.random() < 0.7)  # noqa: E731
        texts += [self.utterance(r, bv).encode() for _ in range(n_customer)]
        import numpy as np
        roles = np.array([synth.ROLE_AGENT] * n_agent + [synth.ROLE_CUSTOMER] * n_customer, dtype=np.uint8)
        lens = np.array([len(t) for t in texts], dtype=np.int64)
        offs = np.zeros(len(texts) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        data = np.frombuffer(b"".join(texts), dtype=np.uint8).copy()
        return synth.Bank(data, offs, roles, texts)

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.cfg, f)


def write_config5(path: str, **kw) -> Config5:
    c = Config5(**kw)
    c.save(path)
    return c


if __name__ == "__main__":
    import sys
    c = Config5()
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/config5.json"
    c.save(out)
    print(out, len(c.custom_names), "custom types;", len(c.cfg["inspect_config"]["rule_set"]), "rule sets")
    assert all(re.compile(x["regex"]["pattern"]) for x in c.cfg["inspect_config"]["custom_info_types"] if "regex" in x)
