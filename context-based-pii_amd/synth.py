"""Synthetic contact-centre transcripts for BASELINE configs 2-4.

Agent rows come from a template bank that mentions the dlp_config.yaml context keywords
(main_service/dlp_config.yaml:5-91) in ~30% of rows; customer rows carry one PII value in ~35% of
rows (validated types half valid, half near-miss), with a hotword phrase 0..80 B before it.

Generating 10M utterances one by one in Python is too slow, so a seeded BANK of unique utterances is
generated per role and the corpus is assembled from bank indices with numpy.  Every corpus row knows
its bank id, which lets parity tests check any sampled row against the CPU oracle.
Lengths: lognormal, mean ~120 B, sigma 0.5, clipped to 8..1024 B.  Seed: PCG64(20250718).
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

SEED = 20250718
ROLE_CUSTOMER, ROLE_AGENT = 0, 1

FILLER = ("thanks okay so well then just one moment please let me check that for you sure right "
          "now sorry hold on perfect great understood certainly of course see here the system shows "
          "it looks like we have your order on file today this morning yesterday again quickly").split()
NAMES = ["jane", "john", "maria", "li", "omar", "sofia", "tom", "ana", "raj", "eva", "kim", "leo"]
DOMAINS = ["example.com", "mail.example.org", "corp.test", "inbox.example.net"]
STREETS = ["Oak", "Maple", "Pine", "Cedar", "Elm", "Lake View", "Sunset", "Hill"]
SUFFIXES = ["Avenue", "Street", "Road", "Boulevard", "Drive", "Lane", "Way", "Court", "Ave", "St"]
CITIES = ["Springfield", "Riverton", "Fairview", "Georgetown", "Salem", "Madison"]
STATES = ["IL", "NY", "CA", "TX", "WA", "OH"]
MONTHS = ["January", "February", "March", "April", "May", "June", "July", "August", "September",
          "October", "November", "December"]
MBI_A = "ACDEFGHJKMNPQRTUVWXY"

AGENT_KEYWORD_TEMPLATES = [
    "Can you please confirm your {kw} for verification?",
    "For our records, could you provide the {kw} on the account?",
    "I will need the {kw} before we continue.",
    "Please read me your {kw} when you are ready.",
]
AGENT_PLAIN = [
    "Thank you for calling, how can I help you today?",
    "Let me look into that for you, one moment please.",
    "I understand, thank you for your patience.",
    "Is there anything else I can help you with?",
    "I have updated the request, you should receive an update soon.",
]
CUSTOMER_PLAIN = [
    "Sure, give me a second to find it.",
    "Okay, that sounds good to me.",
    "I already told the previous person about this.",
    "Thanks, I appreciate the help.",
    "Can you repeat that please?",
]
HOTWORDS = {
    "US_SOCIAL_SECURITY_NUMBER": ["social security", "ssn"], "US_PASSPORT": ["passport"],
    "US_DRIVERS_LICENSE_NUMBER": ["driver's license"], "US_EMPLOYER_IDENTIFICATION_NUMBER": ["ein"],
    "US_MEDICARE_BENEFICIARY_ID_NUMBER": ["mbi", "medicare beneficiary id"], "DOD_ID_NUMBER": ["dod id"],
    "US_INDIVIDUAL_TAXPAYER_IDENTIFICATION_NUMBER": ["itin", "tax id"], "ALIEN_REGISTRATION_NUMBER":
    ["alien registration number"], "BORDER_CROSSING_CARD": ["bcc", "border crossing card"],
    "CREDIT_CARD_NUMBER": ["credit card", "card number"], "FINANCIAL_ACCOUNT_NUMBER": ["account number"],
    "CVV_NUMBER": ["cvv"], "SWIFT_CODE": ["swift code", "bic code"], "IBAN_CODE": ["iban"],
    "PHONE_NUMBER": ["phone number", "contact number"], "EMAIL_ADDRESS": ["email address"],
    "STREET_ADDRESS": ["home address", "address"], "DATE_OF_BIRTH": ["date of birth", "dob"],
    "IMEI_HARDWARE_ID": ["imei"], "MAC_ADDRESS": ["mac address"], "IP_ADDRESS": ["ip address"],
    "SOCIAL_HANDLE": ["handle"],
}


def _luhn_digit(body: str) -> str:
    s = 0
    for i, c in enumerate(reversed(body)):
        x = int(c)
        if i % 2 == 0:
            x *= 2
            if x > 9:
                x -= 9
        s += x
    return str((10 - s % 10) % 10)


def _digits(r, n):
    return "".join(r.choice("0123456789") for _ in range(n))


def _iban(r, valid):
    bban = _digits(r, 18)
    num = int("".join(str(int(c, 36)) for c in bban + "DE00"))
    chk = 98 - num % 97
    if not valid:
        chk = (chk + 1 + r.randrange(90)) % 97 + 2
    return f"DE{chk:02d}{bban}"


def pii_value(r: random.Random, t: str, valid: bool) -> str:
    if t == "EMAIL_ADDRESS":
        return f"{r.choice(NAMES)}.{r.choice(NAMES)}{r.randrange(100)}@{r.choice(DOMAINS)}"
    if t == "PHONE_NUMBER":
        a = str(r.randrange(2, 10)) if valid else str(r.randrange(0, 2))
        num = a + _digits(r, 2), str(r.randrange(2, 10)) + _digits(r, 2), _digits(r, 4)
        return r.choice([f"({num[0]}) {num[1]}-{num[2]}", f"{num[0]}-{num[1]}-{num[2]}", f"{num[0]}.{num[1]}.{num[2]}"])
    if t in ("CREDIT_CARD_NUMBER", "IMEI_HARDWARE_ID"):
        n = 16 if t == "CREDIT_CARD_NUMBER" else 15
        body = r.choice("3456") + _digits(r, n - 2)
        d = _luhn_digit(body)
        if not valid:
            d = str((int(d) + 1 + r.randrange(9)) % 10)
        s = body + d
        if t == "CREDIT_CARD_NUMBER" and r.random() < 0.6:
            sep = r.choice("- ")
            s = sep.join(s[i:i + 4] for i in range(0, 16, 4))
        return s
    if t == "US_PASSPORT":
        return r.choice(["", "E", "C"]) + _digits(r, 9)
    if t == "STREET_ADDRESS":
        return (f"{r.randrange(1, 9999)} {r.choice(STREETS)} {r.choice(SUFFIXES)}, {r.choice(CITIES)}, "
                f"{r.choice(STATES)} {_digits(r, 5)}")
    if t == "US_SOCIAL_SECURITY_NUMBER":
        area = f"{r.randrange(1, 899):03d}" if valid else r.choice(["000", "666", "9" + _digits(r, 2)])
        if area == "666":
            area = "667" if valid else area
        return f"{area}-{r.randrange(1, 100):02d}-{r.randrange(1, 10000):04d}"
    if t == "FINANCIAL_ACCOUNT_NUMBER":
        return _digits(r, r.randrange(8, 18))
    if t == "CVV_NUMBER":
        return _digits(r, r.choice([3, 4]))
    if t == "US_DRIVERS_LICENSE_NUMBER":
        return r.choice("ABCDGKMPSW") + _digits(r, r.randrange(7, 13))
    if t == "US_EMPLOYER_IDENTIFICATION_NUMBER":
        p = r.choice([12, 20, 35, 46, 55, 94]) if valid else r.choice([7, 8, 9, 17, 18, 19, 28, 29, 49])
        return f"{p:02d}-{_digits(r, 7)}"
    if t == "US_MEDICARE_BENEFICIARY_ID_NUMBER":
        a = MBI_A if valid else "SLOIBZ"
        return (f"{r.randrange(1, 10)}{r.choice(a)}{r.choice(MBI_A)}{r.randrange(10)}-{r.choice(MBI_A)}"
                f"{r.choice(MBI_A)}{r.randrange(10)}-{r.choice(MBI_A)}{r.choice(MBI_A)}{_digits(r, 2)}")
    if t == "US_INDIVIDUAL_TAXPAYER_IDENTIFICATION_NUMBER":
        g = r.choice([70, 78, 88, 90, 92, 94, 99]) if valid else r.choice([10, 40, 89, 93])
        return f"9{_digits(r, 2)}-{g}-{_digits(r, 4)}"
    if t == "DOD_ID_NUMBER":
        return _digits(r, 10)
    if t == "MAC_ADDRESS":
        sep = r.choice("-:")
        return sep.join(f"{r.randrange(256):02X}" for _ in range(6 if valid else 5))
    if t == "IP_ADDRESS":
        o = [r.randrange(256) for _ in range(4)]
        if not valid:
            o[r.randrange(4)] = r.randrange(256, 999)
        return ".".join(map(str, o))
    if t == "SWIFT_CODE":
        cc = r.choice(["DE", "US", "GB", "FR"]) if valid else r.choice(["QQ", "XZ", "ZQ"])
        return "".join(r.choice("ABCDEFGHKLMNPRSTUW") for _ in range(4)) + cc + "FF" + r.choice(["", "XXX"])
    if t == "IBAN_CODE":
        return _iban(r, valid)
    if t == "DATE_OF_BIRTH":
        if r.random() < 0.5:
            return f"{r.randrange(1, 13):02d}/{r.randrange(1, 29):02d}/{r.randrange(1940, 2010)}"
        return f"{r.choice(MONTHS)} {r.randrange(1, 29)}, {r.randrange(1940, 2010)}"
    if t == "ALIEN_REGISTRATION_NUMBER":
        return "A" + _digits(r, r.randrange(7, 10))
    if t == "SOCIAL_HANDLE":
        return "@" + r.choice(NAMES).capitalize() + r.choice(["_", ".", ""]) + _digits(r, r.randrange(0, 4))
    if t == "BORDER_CROSSING_CARD":
        return r.choice("BCDXY") + _digits(r, 7)
    raise KeyError(t)


PII_TYPES = list(HOTWORDS.keys())


def _pad(r: random.Random, core: str, target: int) -> str:
    words = []
    n = len(core)
    while n < target:
        w = r.choice(FILLER)
        words.append(w)
        n += len(w) + 1
    if not words:
        return core
    s = core + " " + " ".join(words)
    return s[:max(target, len(core))]


def _keywords():
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rules", "dlp_config.json")
    with open(p) as f:
        kw = json.load(f)["context_keywords"]
    return [k for ks in kw.values() for k in ks]


def _target_len(r: random.Random) -> int:
    return int(min(1024, max(8, round(r.lognormvariate(4.6625, 0.5)))))


def agent_utterance(r: random.Random, keywords) -> str:
    if r.random() < 0.30:
        core = r.choice(AGENT_KEYWORD_TEMPLATES).format(kw=r.choice(keywords))
    else:
        core = r.choice(AGENT_PLAIN)
    return _pad(r, core, _target_len(r))


def customer_utterance(r: random.Random) -> str:
    target = _target_len(r)
    if r.random() < 0.35:
        t = r.choice(PII_TYPES)
        v = pii_value(r, t, r.random() < 0.5)
        gap = " ".join(r.choice(FILLER) for _ in range(r.randrange(0, 12)))
        gap = gap[:r.randrange(0, 81)].strip()
        hw = r.choice(HOTWORDS[t]) if r.random() < 0.8 else "number"
        core = f"My {hw} {gap} is {v}." if gap else f"My {hw} is {v}."
    else:
        core = r.choice(CUSTOMER_PLAIN)
    return _pad(r, core, target)


def agent_bank_sample(n: int, seed: int = SEED) -> List[str]:
    r = random.Random(seed)
    kws = _keywords()
    return [agent_utterance(r, kws) for _ in range(n)]


@dataclass
class Bank:
    data: np.ndarray        # uint8, concatenated utterances
    offsets: np.ndarray     # int64 [n+1]
    roles: np.ndarray       # uint8 [n]
    texts: List[bytes]


def build_bank(n_agent: int = 16384, n_customer: int = 16384, seed: int = SEED) -> Bank:
    r = random.Random(seed)
    kws = _keywords()
    texts = [agent_utterance(r, kws).encode() for _ in range(n_agent)]
    texts += [customer_utterance(r).encode() for _ in range(n_customer)]
    roles = np.array([ROLE_AGENT] * n_agent + [ROLE_CUSTOMER] * n_customer, dtype=np.uint8)
    lens = np.array([len(t) for t in texts], dtype=np.int64)
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(texts), dtype=np.uint8).copy()
    return Bank(data, offs, roles, texts)


@dataclass
class Corpus:
    data: np.ndarray        # uint8 [total bytes]
    offsets: np.ndarray     # uint64 [n+1]
    conv_slot: np.ndarray   # uint32 [n]
    role: np.ndarray        # uint8 [n]
    ts_us: np.ndarray       # int64 [n]
    bank_id: np.ndarray     # int32 [n]

    @property
    def n(self):
        return len(self.role)


@dataclass
class CorpusMeta:
    bank_id: np.ndarray     # int32 [n]
    offsets: np.ndarray     # uint64 [n+1]
    conv_slot: np.ndarray   # uint32 [n]
    role: np.ndarray        # uint8 [n]
    ts_us: np.ndarray       # int64 [n]

    @property
    def n(self):
        return len(self.role)


def corpus_meta(n_conv: int, utt_per_conv: int, bank: Bank, seed: int = SEED, conv_base: int = 0) -> CorpusMeta:
    """Conversation-major layout: conversation c's rows are contiguous and in entry order,
    alternating AGENT / END_USER, 5 s apart (the batch contract of include/pii_engine.h)."""
    g = np.random.Generator(np.random.PCG64(seed + conv_base))
    n = n_conv * utt_per_conv
    n_agent = int((bank.roles == ROLE_AGENT).sum())
    n_cust = len(bank.roles) - n_agent
    pos = np.tile(np.arange(utt_per_conv), n_conv)
    role = (pos % 2 == 0).astype(np.uint8)          # even entries: AGENT
    bid = np.where(role == ROLE_AGENT, g.integers(0, n_agent, n), n_agent + g.integers(0, n_cust, n))
    bid = bid.astype(np.int32)
    lens = (bank.offsets[1:] - bank.offsets[:-1])[bid]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    conv = (np.repeat(np.arange(n_conv, dtype=np.uint32), utt_per_conv) + np.uint32(conv_base)).astype(np.uint32)
    ts = (1_760_000_000_000_000 + pos.astype(np.int64) * 5_000_000).astype(np.int64)
    return CorpusMeta(bid, offs, conv, role, ts)


def gather_bytes(meta: CorpusMeta, bank: Bank, lo: int = 0, hi: int = None) -> np.ndarray:
    """Bytes of rows [lo, hi) (numpy; use for small corpora or samples)."""
    hi = meta.n if hi is None else hi
    bid = meta.bank_id[lo:hi]
    lens = (bank.offsets[1:] - bank.offsets[:-1])[bid]
    total = int(lens.sum())
    out_off = np.zeros(len(bid) + 1, dtype=np.int64)
    np.cumsum(lens, out=out_off[1:])
    rep = np.repeat(bank.offsets[:-1][bid].astype(np.int64) - out_off[:-1], lens)
    return bank.data[np.arange(total, dtype=np.int64) + rep]


def make_corpus(n_conv: int, utt_per_conv: int, bank: Bank, seed: int = SEED, conv_base: int = 0) -> Corpus:
    m = corpus_meta(n_conv, utt_per_conv, bank, seed, conv_base)
    return Corpus(gather_bytes(m, bank), m.offsets, m.conv_slot, m.role, m.ts_us, m.bank_id)


def reorder(meta: CorpusMeta, bank: Bank, perm: np.ndarray) -> CorpusMeta:
    """rows of `meta` in the order `perm` (offsets recomputed)"""
    bid = meta.bank_id[perm]
    lens = (bank.offsets[1:] - bank.offsets[:-1])[bid]
    offs = np.zeros(len(bid) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return CorpusMeta(bid, offs, meta.conv_slot[perm], meta.role[perm], meta.ts_us[perm])


def stream_order(n_conv: int, utt_per_conv: int, steps_per_batch: int) -> Tuple[np.ndarray, List[Tuple[int, int]]]:
    """Config 4 stream order of a conversation-major corpus: batch b carries steps
    [b*s, (b+1)*s) of every conversation (a conversation's rows spread over all batches), and inside
    a batch a conversation's rows are contiguous (the engine's batch contract).  Returns the row
    permutation and the [lo, hi) row range of every batch."""
    perm, ranges, lo = [], [], 0
    for k0 in range(0, utt_per_conv, steps_per_batch):
        k1 = min(utt_per_conv, k0 + steps_per_batch)
        p = (np.arange(n_conv, dtype=np.int64)[:, None] * utt_per_conv + np.arange(k0, k1)[None, :]).reshape(-1)
        perm.append(p)
        ranges.append((lo, lo + len(p)))
        lo += len(p)
    return np.concatenate(perm), ranges


def step_major(meta: CorpusMeta, bank: Bank, n_conv: int, utt_per_conv: int) -> CorpusMeta:
    """The same rows streamed the way the aggregator sees them (config 3): step k = the k-th
    utterance of every conversation, so rows [k*n_conv, (k+1)*n_conv) are one re-scan call."""
    perm = (np.arange(utt_per_conv)[:, None] + utt_per_conv * np.arange(n_conv)[None, :]).reshape(-1)
    bid = meta.bank_id[perm]
    lens = (bank.offsets[1:] - bank.offsets[:-1])[bid]
    offs = np.zeros(len(bid) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    return CorpusMeta(bid, offs, meta.conv_slot[perm], meta.role[perm], meta.ts_us[perm])
