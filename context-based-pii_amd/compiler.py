"""Host rule compiler: dlp_config.yaml (+ build-defined built-ins) -> DFA tables -> rules blob.

Replaces what Google Cloud DLP does internally with ``inspect_config`` (dlp_config.yaml:92-194) and
with the context branch of ``call_dlp_for_redaction`` (main_service/main.py:609-686).

Regexes are parsed with the standard library's own ``sre_parse`` (the parser ``re`` uses), as BYTES
patterns, so the engine and the CPU oracle start from the same syntax tree.  Three DFA families are
built from a Thompson NFA with explicit assertion nodes (``\\b``, ``\\B``, ``\\A``/``^``, ``\\Z``):

* SCAN   - one REVERSE, unanchored, set-semantics DFA over every detector pattern and every
           context-keyword group.  The HIP scan kernel walks each utterance right-to-left through it;
           entering a state whose accept list is non-empty means "a match of these patterns STARTS
           here".  It is the only dense, per-byte table (LDS-resident).
* FIRST  - per detector pattern, an ANCHORED leftmost-first (priority-ordered, RE2-style) forward
           DFA.  Run from a start found by SCAN it returns exactly the end ``re`` would return.
* HOT    - per hotword rule, an unanchored set-semantics forward DFA run over the proximity window
           (window edges behave as text edges, like ``re.search(text[lo:hi])``).

Assertions are resolved with one character of look-ahead: a DFA state is (core NFA set, kind of the
previous character); closures are taken with the kind of the NEXT character known, so acceptance is
reported one step late, as a property of the state entered (see DESIGN.md §DFA encoding).
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import dataclasses
import re
import struct
import sys
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import yaml

if sys.version_info >= (3, 11):                               # pragma: no cover
    from re import _constants as C
    from re import _parser as sre_parse
else:
    import sre_constants as C
    import sre_parse

HERE = os.path.dirname(os.path.abspath(__file__))
RULES_DIR = os.path.join(HERE, "rules")

LIKELIHOOD = {"LIKELIHOOD_UNSPECIFIED": 0, "VERY_UNLIKELY": 1, "UNLIKELY": 2, "POSSIBLE": 3,
              "LIKELY": 4, "VERY_LIKELY": 5}
VERY_LIKELY = 5
DEFAULT_MIN_LIKELIHOOD = 3
VALIDATOR_IDS = {None: 0, "luhn": 1, "nanp": 2, "ssn": 3, "ein": 4, "ipv4": 5, "swift": 6, "iban": 7}
BLOB_MAGIC = b"PIIRULE1"
PSEUDO_GROUP_MAX_TYPES = 64     # rule sets up to this many types get a context variant per type


class RuleError(ValueError):
    pass


def lik_value(x) -> int:
    return x if isinstance(x, int) else LIKELIHOOD[str(x)]


# ============================================================================ character sets ====
ALL = (1 << 256) - 1
DIGIT = sum(1 << c for c in range(48, 58))
WORD = DIGIT | sum(1 << c for c in range(65, 91)) | sum(1 << c for c in range(97, 123)) | (1 << 95)
SPACE = sum(1 << c for c in (9, 10, 11, 12, 13, 32))
NEWLINE = 1 << 10
UPPER = sum(1 << c for c in range(65, 91))
LOWER = sum(1 << c for c in range(97, 123))


def fold(cs: int) -> int:
    """ASCII case closure (IGNORECASE on bytes patterns)."""
    return cs | ((cs & UPPER) << 32) | ((cs & LOWER) >> 32)


_CATEGORIES = {
    C.CATEGORY_DIGIT: DIGIT, C.CATEGORY_NOT_DIGIT: ALL & ~DIGIT,
    C.CATEGORY_WORD: WORD, C.CATEGORY_NOT_WORD: ALL & ~WORD,
    C.CATEGORY_SPACE: SPACE, C.CATEGORY_NOT_SPACE: ALL & ~SPACE,
}

# assertion kinds (forward sense); the reverse NFA swaps BEGIN <-> END
A_BOUNDARY, A_NONBOUNDARY, A_BEGIN, A_END = range(4)
# character kinds: BOT (no previous char), W word char, N non-word char, EOT (no next char)
K_BOT, K_W, K_N, K_EOT = 0, 1, 2, 3


def assert_ok(kind: int, pk: int, nk: int) -> bool:
    if kind == A_BOUNDARY or kind == A_NONBOUNDARY:
        b = (pk == K_W) != (nk == K_W)
        return b if kind == A_BOUNDARY else not b
    if kind == A_BEGIN:
        return pk == K_BOT
    return nk == K_EOT


# ======================================================================================= NFA ====
CHAR, SPLIT, EPS, ASSERT, MATCH = range(5)


class NFA:
    def __init__(self):
        self.kind: List[int] = []
        self.a: List[int] = []      # CHAR/EPS/ASSERT: next ; SPLIT: preferred ; MATCH: pattern id
        self.b: List[int] = []      # SPLIT: other ; ASSERT: assertion kind
        self.cs: List[int] = []     # CHAR: byte set

    def add(self, kind, a=-1, b=-1, cs=0) -> int:
        self.kind.append(kind)
        self.a.append(a)
        self.b.append(b)
        self.cs.append(cs)
        return len(self.kind) - 1


def parse(pattern: str):
    try:
        return sre_parse.parse(pattern.encode("ascii") if isinstance(pattern, str) else pattern, 0)
    except Exception as e:  # pragma: no cover - surfaced to the caller
        raise RuleError(f"cannot parse regex {pattern!r}: {e}")


def _items_nullable(items) -> bool:
    return all(_nullable(op, av) for op, av in items)


def _nullable(op, av) -> bool:
    if op in (C.LITERAL, C.NOT_LITERAL, C.ANY, C.IN):
        return False
    if op == C.AT:
        return True
    if op == C.SUBPATTERN:
        return _items_nullable(av[-1])
    if op == C.BRANCH:
        return any(_items_nullable(b) for b in av[1])
    if op in (C.MAX_REPEAT, C.MIN_REPEAT):
        return av[0] == 0 or _items_nullable(av[2])
    raise RuleError(f"unsupported regex construct {op}")


class Emitter:
    """Thompson construction by continuation: emit(items, cont) returns the entry node."""

    def __init__(self, nfa: NFA, reverse: bool):
        self.nfa = nfa
        self.reverse = reverse

    def charset(self, op, av, flags) -> int:
        ic = flags & C.SRE_FLAG_IGNORECASE
        if op == C.LITERAL:
            cs = 1 << av
            return fold(cs) if ic else cs
        if op == C.NOT_LITERAL:
            cs = 1 << av
            return ALL & ~(fold(cs) if ic else cs)
        if op == C.ANY:
            return ALL if flags & C.SRE_FLAG_DOTALL else ALL & ~NEWLINE
        if op == C.IN:
            cs, neg = 0, False
            for iop, iav in av:
                if iop == C.NEGATE:
                    neg = True
                elif iop == C.LITERAL:
                    cs |= 1 << iav
                elif iop == C.RANGE:
                    lo, hi = iav
                    cs |= ((1 << (hi + 1)) - 1) & ~((1 << lo) - 1)
                elif iop == C.CATEGORY:
                    cs |= _CATEGORIES[iav]
                else:
                    raise RuleError(f"unsupported class item {iop}")
            if ic:
                cs = fold(cs)
            return (ALL & ~cs) if neg else cs
        raise AssertionError(op)

    def emit(self, items, flags, cont) -> int:
        seq = list(items)
        if not self.reverse:
            seq = seq[::-1]
        for op, av in seq:          # build back to front: each item continues into `cont`
            cont = self.emit_one(op, av, flags, cont)
        return cont

    def emit_one(self, op, av, flags, cont) -> int:
        n = self.nfa
        if op in (C.LITERAL, C.NOT_LITERAL, C.ANY, C.IN):
            return n.add(CHAR, cont, cs=self.charset(op, av, flags))
        if op == C.SUBPATTERN:
            _group, add_f, del_f, sub = av
            if add_f & C.SRE_FLAG_MULTILINE:
                raise RuleError("MULTILINE is not supported")
            return self.emit(sub, (flags | add_f) & ~del_f, cont)
        if op == C.BRANCH:
            alts = [self.emit(b, flags, cont) for b in av[1]]
            entry = alts[-1]
            for alt in reversed(alts[:-1]):
                entry = n.add(SPLIT, alt, entry)
            return entry
        if op in (C.MAX_REPEAT, C.MIN_REPEAT):
            lo, hi, sub = av
            greedy = op == C.MAX_REPEAT
            if _items_nullable(sub) and hi != lo:
                raise RuleError("repeat of a sub-pattern that can match empty is not supported")
            if hi == C.MAXREPEAT:
                loop = n.add(SPLIT)
                body = self.emit(sub, flags, loop)
                if greedy:
                    n.a[loop], n.b[loop] = body, cont
                else:
                    n.a[loop], n.b[loop] = cont, body
                tail = loop
            else:
                tail = cont
                for _ in range(hi - lo):
                    body = self.emit(sub, flags, tail)
                    tail = n.add(SPLIT, body, cont) if greedy else n.add(SPLIT, cont, body)
            for _ in range(lo):
                tail = self.emit(sub, flags, tail)
            return tail
        if op == C.AT:
            if av in (C.AT_BOUNDARY,):
                k = A_BOUNDARY
            elif av == C.AT_NON_BOUNDARY:
                k = A_NONBOUNDARY
            elif av in (C.AT_BEGINNING, C.AT_BEGINNING_STRING):
                k = A_BEGIN
            elif av == C.AT_END_STRING:
                k = A_END
            else:
                raise RuleError("'$' / MULTILINE anchors are not supported (use \\Z)")
            if self.reverse and k in (A_BEGIN, A_END):
                k = A_END if k == A_BEGIN else A_BEGIN
            return n.add(ASSERT, cont, k)
        raise RuleError(f"unsupported regex construct {op}")


def add_pattern(nfa: NFA, pattern: str, pid: int, reverse: bool) -> int:
    tree = parse(pattern)
    flags = tree.state.flags
    if flags & C.SRE_FLAG_MULTILINE:
        raise RuleError("MULTILINE is not supported")
    if _items_nullable(list(tree)):
        raise RuleError(f"pattern {pattern!r} can match the empty string")
    m = nfa.add(MATCH, pid)
    return Emitter(nfa, reverse).emit(list(tree), flags, m)


# ================================================================================ byte classes ==
def byte_classes(nfa: NFA) -> Tuple[np.ndarray, List[int]]:
    """Coarsest partition of 0..255 respecting every CHAR set and the word-character set."""
    blocks = [ALL]
    sets = {WORD, NEWLINE}
    sets.update(cs for k, cs in zip(nfa.kind, nfa.cs) if k == CHAR)
    for s in sets:
        nb = []
        for b in blocks:
            x, y = b & s, b & ~s
            if x:
                nb.append(x)
            if y:
                nb.append(y)
        blocks = nb
    cmap = np.zeros(256, dtype=np.uint8)
    reps = []
    blocks.sort(key=lambda b: (b & -b).bit_length())   # order classes by smallest member
    for ci, b in enumerate(blocks):
        reps.append((b & -b).bit_length() - 1)
        for c in range(256):
            if (b >> c) & 1:
                cmap[c] = ci
    if len(blocks) > 255:
        raise RuleError("too many byte classes")
    return cmap, reps


def _kind_of_byte(c: int) -> int:
    return K_W if (WORD >> c) & 1 else K_N


# ================================================================================== DFA core ====
@dataclass
class DFA:
    cmap: np.ndarray                 # uint8[256] byte -> class
    trans: np.ndarray                # uint16[S, C+1]; column C = end-of-text pseudo-class
    flags: np.ndarray                # uint8[S]
    start: List[int]                 # start state per previous-character kind (BOT, W, N)
    accept: List[Tuple[int, ...]] = field(default_factory=list)   # set DFAs: pattern ids per state

    @property
    def n_states(self):
        return self.trans.shape[0]

    @property
    def n_classes(self):
        return self.trans.shape[1] - 1


def _closure_set(nfa: NFA, seeds, pk, nk):
    kind, a, b = nfa.kind, nfa.a, nfa.b
    chars, matches, seen, stack = [], [], set(), list(seeds)
    while stack:
        s = stack.pop()
        if s in seen:
            continue
        seen.add(s)
        k = kind[s]
        if k == CHAR:
            chars.append(s)
        elif k == MATCH:
            matches.append(a[s])
        elif k == SPLIT:
            stack.append(a[s])
            stack.append(b[s])
        elif k == EPS:
            stack.append(a[s])
        elif assert_ok(b[s], pk, nk):
            stack.append(a[s])
    return chars, frozenset(matches)


def _closure_ordered(nfa: NFA, seeds, pk, nk):
    kind, a, b = nfa.kind, nfa.a, nfa.b
    out, seen = [], set()
    for seed in seeds:
        stack = [seed]
        while stack:
            s = stack.pop()
            if s in seen:
                continue
            seen.add(s)
            k = kind[s]
            if k == CHAR or k == MATCH:
                out.append(s)
            elif k == SPLIT:
                stack.append(b[s])          # lower priority explored after the preferred branch
                stack.append(a[s])
            elif k == EPS:
                stack.append(a[s])
            elif assert_ok(b[s], pk, nk):
                stack.append(a[s])
    return out


def build_set_dfa(nfa: NFA, starts: Sequence[int], unanchored: bool, max_states: int = 60000) -> DFA:
    """Set-semantics DFA.  State key = (core, prev kind, accept set); accept set = patterns whose
    match ENDS right before the character just consumed (reported one step late)."""
    cmap, reps = byte_classes(nfa)
    ncls = len(reps)
    ckind = [_kind_of_byte(r) for r in reps]
    start_set = frozenset(starts)
    index: Dict[tuple, int] = {}
    keys: List[tuple] = []

    def sid(key):
        if key not in index:
            if len(keys) >= max_states:
                raise RuleError(f"DFA exceeds {max_states} states")
            index[key] = len(keys)
            keys.append(key)
        return index[key]

    empty = frozenset()
    starts_by_kind = []
    for pk in (K_BOT, K_W, K_N):
        starts_by_kind.append(sid((empty if unanchored else start_set, pk, empty)))
    rows = []
    i = 0
    while i < len(keys):
        core, pk, _acc = keys[i]
        row = [0] * (ncls + 1)
        seeds = (core | start_set) if unanchored else core
        if not seeds:                                    # anchored dead state
            row = [i] * (ncls + 1)
            rows.append(row)
            i += 1
            continue
        clos = {}
        for nk in (K_W, K_N, K_EOT):
            clos[nk] = _closure_set(nfa, seeds, pk, nk)
        for c in range(ncls):
            chars, acc = clos[ckind[c]]
            r = reps[c]
            nxt = frozenset(nfa.a[s] for s in chars if (nfa.cs[s] >> r) & 1)
            if not unanchored and not nxt:
                key = (empty, K_N, acc)
            else:
                key = (nxt, ckind[c], acc)
            row[c] = sid(key)
        _, acc = clos[K_EOT]
        row[ncls] = sid((empty, K_EOT, acc))
        rows.append(row)
        i += 1
    trans = np.array(rows, dtype=np.int64)
    accept = [tuple(sorted(k[2])) for k in keys]
    flags = np.array([1 if acc else 0 for acc in accept], dtype=np.uint8)
    dfa = DFA(cmap, trans, flags, starts_by_kind, accept)
    return minimize(dfa)


def relax_items(items, budget: int):
    """Prefix relaxation for the SCAN prefilter: a pattern whose language, for every match of the
    original starting at s, has a match starting at s too (so SCAN reports a SUPERSET of starts;
    the exact FIRST DFA confirms each).  Bounded repeats are widened ({lo,hi} -> {min(lo,k)} X*),
    the sequence is cut after `budget` consuming characters, an alternation ends the prefix."""
    out = []
    for i, (op, av) in enumerate(items):
        if op == C.AT:
            out.append((op, av))
            continue
        if budget <= 0:
            return out, False, 0
        if op in (C.LITERAL, C.NOT_LITERAL, C.ANY, C.IN):
            out.append((op, av))
            budget -= 1
            continue
        if op == C.SUBPATTERN:
            sub, full, budget = relax_items(list(av[-1]), budget)
            out.append((op, (av[0], av[1], av[2], sub)))
            if not full:
                return out, False, 0
            continue
        if op == C.BRANCH:
            # each alternative relaxed with the budget left; when every one of them is taken whole, the
            # prefix goes on past the alternation (with the smallest budget any alternative left), so a
            # pattern like (0?[1-9]|1[0-2])/... keeps its '/' instead of firing at every number
            rs = [relax_items(list(b), budget) for b in av[1]]
            out.append((op, (None, [r[0] for r in rs])))
            if not all(r[1] for r in rs):
                return out, False, 0
            budget = min(r[2] for r in rs)
            continue
        if op in (C.MAX_REPEAT, C.MIN_REPEAT):
            lo, hi, sub = av
            sub = list(sub)
            single = len(sub) == 1 and sub[0][0] in (C.LITERAL, C.NOT_LITERAL, C.ANY, C.IN)
            if not single:
                if lo == 0:
                    return out, False, 0
                for _ in range(lo):
                    s2, full, budget = relax_items(sub, budget)
                    out.extend(s2)
                    if not full:
                        return out, False, 0
                if hi != lo:
                    return out, False, 0
                continue
            if hi != lo and hi != C.MAXREPEAT and hi <= budget and all(o == C.AT for o, _ in items[i + 1:]):
                # a bounded repeat that ends the sequence and fits whole is kept exact, so the trailing
                # assertion still filters -- \b\d{3,4}\b no longer fires at every longer digit run
                # (inside a sequence, widening spends only `lo` of the budget on it: more of what
                # follows is kept, e.g. IP_ADDRESS's dots)
                out.extend(sub * lo)
                out.append((C.MAX_REPEAT, (0, hi - lo, sub)))
                budget -= hi
                continue
            n = min(lo, budget)
            out.extend(sub * n)
            budget -= n
            if n < lo:
                return out, False, 0
            if hi != lo:
                out.append((C.MAX_REPEAT, (0, C.MAXREPEAT, sub)))
            continue
        raise RuleError(f"unsupported regex construct {op}")
    return out, True, budget


def add_relaxed(nfa: NFA, pattern: str, pid: int, budget: int, reverse: bool) -> int:
    tree = parse(pattern)
    items = list(tree)
    if budget > 0:
        items = relax_items(items, budget)[0]
    if _items_nullable(items):
        raise RuleError(f"relaxed pattern of {pattern!r} can match the empty string")
    m = nfa.add(MATCH, pid)
    return Emitter(nfa, reverse).emit(items, tree.state.flags, m)


@dataclass
class MealyDFA:
    cmap: np.ndarray          # uint8[256]
    trans: np.ndarray         # uint16[S, C+1]; bit 15 set = this transition reports accepts
    start: int                # state at the right end of an utterance (reverse scan)
    acc_id: np.ndarray        # int32[S, C+1]: index into acc_sets (0 = none)
    acc_sets: List[Tuple[int, ...]]

    @property
    def n_states(self):
        return self.trans.shape[0]

    @property
    def n_classes(self):
        return self.trans.shape[1] - 1


def build_mealy_dfa(nfa: NFA, starts: Sequence[int], max_states: int = 32767,
                    max_bytes: Optional[int] = None) -> MealyDFA:
    """Unanchored set-semantics DFA with accepts on TRANSITIONS.  Transition (q, c) reports the
    patterns whose match ends right before c in scan direction (for the reverse SCAN: whose match
    STARTS right after c in text order).  `max_bytes` bounds the u16 table (rows padded to an even
    class count) and fails early (RuleError) when the subset construction exceeds it."""
    cmap, reps = byte_classes(nfa)
    ncls = len(reps)
    if max_bytes is not None:
        max_states = min(max_states, max_bytes // (2 * ((ncls + 2) & ~1)) * 2)
    ckind = [_kind_of_byte(r) for r in reps]
    start_set = frozenset(starts)
    index: Dict[tuple, int] = {}
    keys: List[tuple] = []

    def sid(key):
        if key not in index:
            if len(keys) >= max_states:
                raise RuleError(f"SCAN DFA exceeds {max_states} states")
            index[key] = len(keys)
            keys.append(key)
        return index[key]

    sid((frozenset(), K_BOT))
    acc_index: Dict[frozenset, int] = {frozenset(): 0}
    acc_sets: List[Tuple[int, ...]] = [()]
    rows, arows = [], []
    i = 0
    while i < len(keys):
        core, pk = keys[i]
        seeds = core | start_set
        clos = {nk: _closure_set(nfa, seeds, pk, nk) for nk in (K_W, K_N, K_EOT)}
        row, arow = [0] * (ncls + 1), [0] * (ncls + 1)
        for c in range(ncls + 1):
            if c == ncls:
                chars, acc = clos[K_EOT]
                row[c] = sid((frozenset(), K_EOT))
            else:
                chars, acc = clos[ckind[c]]
                r = reps[c]
                row[c] = sid((frozenset(nfa.a[s] for s in chars if (nfa.cs[s] >> r) & 1), ckind[c]))
            if acc:
                if acc not in acc_index:
                    acc_index[acc] = len(acc_sets)
                    acc_sets.append(tuple(sorted(acc)))
                arow[c] = acc_index[acc]
        rows.append(row)
        arows.append(arow)
        i += 1
    trans = np.array(rows, dtype=np.int64)
    accid = np.array(arows, dtype=np.int64)
    # Moore-style refinement on (target block, accept id) per column
    block = np.zeros(len(keys), dtype=np.int64)
    nblocks = 1
    while True:
        sig = np.concatenate([block[:, None], block[trans], accid], axis=1)
        _, nb = np.unique(sig, axis=0, return_inverse=True)
        nb = nb.reshape(-1)
        n = int(nb.max()) + 1
        if n == nblocks:
            break
        block, nblocks = nb, n
    rep = {}
    for s in range(len(keys)):
        rep.setdefault(int(block[s]), s)
    order = sorted(rep.keys(), key=lambda b: rep[b])
    newid = {b: j for j, b in enumerate(order)}
    t2 = np.zeros((nblocks, ncls + 1), dtype=np.uint16)
    a2 = np.zeros((nblocks, ncls + 1), dtype=np.int32)
    for b in order:
        s = rep[b]
        j = newid[b]
        t2[j] = [newid[int(block[t])] for t in trans[s]]
        a2[j] = accid[s]
    if nblocks >= 32768:
        raise RuleError("SCAN DFA too large for 15-bit state ids")
    t2 = t2 | np.where(a2 > 0, 0x8000, 0).astype(np.uint16)
    return MealyDFA(cmap, t2, newid[int(block[0])], a2, acc_sets)


def build_first_dfa(nfa: NFA, start: int, max_states: int = 60000) -> DFA:
    """Anchored leftmost-first DFA (RE2 'first match' construction).  flags bit0: a match ended
    right before the character just consumed; bit1: terminal (no thread left)."""
    cmap, reps = byte_classes(nfa)
    ncls = len(reps)
    ckind = [_kind_of_byte(r) for r in reps]
    index: Dict[tuple, int] = {}
    keys: List[tuple] = []

    def sid(key):
        if key not in index:
            if len(keys) >= max_states:
                raise RuleError(f"DFA exceeds {max_states} states")
            index[key] = len(keys)
            keys.append(key)
        return index[key]

    starts_by_kind = [sid(((start,), pk, 0)) for pk in (K_BOT, K_W, K_N)]
    rows = []
    i = 0
    while i < len(keys):
        core, pk, _m = keys[i]
        row = [0] * (ncls + 1)
        if not core:
            rows.append([i] * (ncls + 1))
            i += 1
            continue
        clos = {}
        for nk in (K_W, K_N, K_EOT):
            leaves = _closure_ordered(nfa, core, pk, nk)
            m = 0
            for j, s in enumerate(leaves):
                if nfa.kind[s] == MATCH:
                    leaves = leaves[:j]
                    m = 1
                    break
            clos[nk] = (leaves, m)
        for c in range(ncls):
            leaves, m = clos[ckind[c]]
            r = reps[c]
            nxt, seen = [], set()
            for s in leaves:
                if (nfa.cs[s] >> r) & 1:
                    t = nfa.a[s]
                    if t not in seen:
                        seen.add(t)
                        nxt.append(t)
            row[c] = sid((tuple(nxt), ckind[c] if nxt else K_N, m))
        leaves, m = clos[K_EOT]
        row[ncls] = sid(((), K_N, m))
        rows.append(row)
        i += 1
    trans = np.array(rows, dtype=np.int64)
    flags = np.array([(k[2] & 1) | (2 if not k[0] else 0) for k in keys], dtype=np.uint8)
    dfa = DFA(cmap, trans, flags, starts_by_kind, [])
    return minimize(dfa)


def minimize(dfa: DFA) -> DFA:
    """Moore partition refinement; initial blocks split by (flags, accept set)."""
    S = dfa.n_states
    if dfa.accept:
        sig0 = [(int(f), acc) for f, acc in zip(dfa.flags, dfa.accept)]
    else:
        sig0 = [(int(f),) for f in dfa.flags]
    uniq = {}
    block = np.array([uniq.setdefault(s, len(uniq)) for s in sig0], dtype=np.int64)
    nblocks = len(uniq)
    while True:
        sig = np.concatenate([block[:, None], block[dfa.trans]], axis=1)
        _, nb = np.unique(sig, axis=0, return_inverse=True)
        nb = nb.reshape(-1)
        n = int(nb.max()) + 1
        if n == nblocks:
            break
        block, nblocks = nb, n
    # renumber: keep start states first (stable), flagged states last (threshold test in kernels)
    rep = {}
    for s in range(S):
        rep.setdefault(int(block[s]), s)
    order = sorted(rep.keys(), key=lambda b: (1 if dfa.flags[rep[b]] else 0, rep[b]))
    newid = {b: i for i, b in enumerate(order)}
    trans = np.zeros((nblocks, dfa.trans.shape[1]), dtype=np.uint16)
    flags = np.zeros(nblocks, dtype=np.uint8)
    accept = [()] * nblocks if dfa.accept else []
    for b in order:
        s = rep[b]
        i = newid[b]
        trans[i] = [newid[int(block[t])] for t in dfa.trans[s]]
        flags[i] = dfa.flags[s]
        if dfa.accept:
            accept[i] = dfa.accept[s]
    start = [newid[int(block[s])] for s in dfa.start]
    if nblocks > 65535:
        raise RuleError("DFA too large for 16-bit state ids")
    return DFA(dfa.cmap, trans, flags, start, accept)


# ================================================================================ rule model ====
@dataclass
class Pattern:
    pid: int
    type_name: str
    pattern: str
    likelihood: int
    validator: Optional[str]
    custom: bool
    scan_prefix: Optional[int] = None     # characters the SCAN prefilter keeps (None: SCAN_BUDGET)


@dataclass
class HotRule:
    pattern: str
    window_before: int
    window_after: int
    fixed: int               # 0 = use relative
    relative: int


class Rules:
    """The rule model both the engine blob and the docs are generated from."""

    def __init__(self, dlp_config: dict, builtin: dict):
        insp = dlp_config.get("inspect_config", {}) or {}
        self.raw = dlp_config
        self.base_info_types = [it.get("name") for it in insp.get("info_types", [])]
        self.custom_defs = list(insp.get("custom_info_types", []) or [])
        self.custom_names = [c.get("info_type", {}).get("name") for c in self.custom_defs]
        self.context_keywords: "OrderedDict[str, list]" = OrderedDict(dlp_config.get("context_keywords", {}) or {})
        dets = builtin["detectors"]
        order = []
        for n in self.base_info_types + self.custom_names + list(dets.keys()) + list(self.context_keywords):
            if n not in order:
                order.append(n)
        # types of external detectors (the NER): last in the type order, no pattern, no variant
        self.external_types = [n for n in (builtin.get("external_types") or []) if n not in order]
        order += self.external_types
        self.type_names = order
        self.type_id = {n: i for i, n in enumerate(order)}
        self.patterns: List[Pattern] = []
        for name, variants in dets.items():
            if name in self.custom_names:
                continue
            for v in variants:
                self.patterns.append(Pattern(len(self.patterns), name, v["pattern"],
                                             lik_value(v.get("likelihood", "POSSIBLE")), v.get("validator"), False,
                                             v.get("scan_prefix")))
        for c in self.custom_defs:
            name = c["info_type"]["name"]
            if "regex" in c:
                pat = c["regex"]["pattern"]
            elif "dictionary" in c:
                words = c["dictionary"]["word_list"]["words"]
                pat = r"(?i)\b(?:" + "|".join(re.escape(w) for w in words) + r")\b"
            else:
                raise RuleError(f"unsupported custom infoType {name}")
            # dictionary words: a 3-character prefix fires at most word starts of ordinary text (13x the
            # matches on config 5's text), a 4-character one about 1.5x (SCAN prefilter, see plan_scan_groups)
            self.patterns.append(Pattern(len(self.patterns), name, pat,
                                         lik_value(c.get("likelihood", "VERY_LIKELY")), None, True,
                                         DICT_SCAN_PREFIX if "dictionary" in c else None))
        for p in self.patterns:
            if p.validator not in VALIDATOR_IDS:
                raise RuleError(f"unknown validator {p.validator}")
        # context keyword groups (main.py:558-578): group g -> (type, regex or None, always-hit)
        self.kw_groups = []
        for t, kws in self.context_keywords.items():
            kws = [str(k) for k in (kws or [])]
            always = any(k == "" for k in kws)
            usable = [k for k in kws if k and k == k.lower()]   # upper-case keywords never hit lower()ed text
            pat = "(?i)(?:" + "|".join(re.escape(k) for k in usable) + ")" if usable else None
            self.kw_groups.append((t, pat, always))
        # Every other info type becomes a keyword-less context group, so that a context record naming
        # it (call_dlp_for_redaction(transcript, {"expected_pii_type": t}), main.py:614-686) has a
        # compiled variant.  extract_expected_pii never returns one (no keywords).  Large rule sets
        # (config 5) skip this: V * T variant tables would not fit the kernels' LDS images.
        self.n_keyword_groups = len(self.kw_groups)
        if len(self.type_names) <= PSEUDO_GROUP_MAX_TYPES:
            named = {t for t, _, _ in self.kw_groups} | set(self.external_types)
            self.kw_groups.extend((t, None, False) for t in self.type_names if t not in named)

    @classmethod
    def load(cls, dlp_config_path: Optional[str] = None, builtin_path: Optional[str] = None) -> "Rules":
        dlp_config_path = dlp_config_path or os.path.join(RULES_DIR, "dlp_config.json")
        builtin_path = builtin_path or os.path.join(RULES_DIR, "builtin_infotypes.yaml")
        with open(dlp_config_path) as f:
            cfg = json.load(f) if dlp_config_path.endswith(".json") else yaml.safe_load(f)
        with open(builtin_path) as f:
            builtin = yaml.safe_load(f)
        return cls(cfg, builtin)

    # ---- a6, main.py:609-686, restated statelessly -------------------------------
    def merged_inspect_config(self, expected_type: Optional[str]) -> dict:
        import copy
        cfg = copy.deepcopy(self.raw.get("inspect_config", {}) or {})
        if not expected_type:
            return cfg
        custom = next((c for c in self.custom_defs if c.get("info_type", {}).get("name") == expected_type), None)
        if custom is not None:
            cfg.setdefault("custom_info_types", [])
            if expected_type not in {c.get("info_type", {}).get("name") for c in cfg["custom_info_types"]}:
                cfg["custom_info_types"].append(copy.deepcopy(custom))
            return cfg
        cfg.setdefault("info_types", [])
        if expected_type not in {it.get("name") for it in cfg["info_types"]}:
            cfg["info_types"].append({"name": expected_type})
        cfg.setdefault("rule_set", [])
        found = False
        for entry in cfg["rule_set"]:
            if "info_types" in entry and expected_type in {it.get("name") for it in entry["info_types"]}:
                for rule in entry.get("rules", []):
                    if "hotword_rule" in rule and "likelihood_adjustment" in rule["hotword_rule"]:
                        rule["hotword_rule"]["likelihood_adjustment"]["fixed_likelihood"] = VERY_LIKELY
                        found = True
                        break
                if found:
                    break
        if not found:
            cfg["rule_set"].append({"info_types": [{"name": expected_type}], "rules": [{"hotword_rule": {
                "hotword_regex": {"pattern": ".+"}, "proximity": {"window_before": 100, "window_after": 100},
                "likelihood_adjustment": {"fixed_likelihood": VERY_LIKELY}}}]})
        return cfg

    def variants(self):
        """Variant 0 = no context; variant 1+g = expected type of keyword group g."""
        out = [self.merged_inspect_config(None)]
        for t, _, _ in self.kw_groups:
            out.append(self.merged_inspect_config(t))
        return out


# =================================================================================== blob =======
_DT = {np.dtype(np.uint8): 1, np.dtype(np.uint16): 2, np.dtype(np.uint32): 3, np.dtype(np.int32): 4,
       np.dtype(np.int64): 5, np.dtype(np.int8): 6}


def _sections_to_blob(sections: "OrderedDict[str, np.ndarray]") -> bytes:
    out = io.BytesIO()
    out.write(BLOB_MAGIC)
    out.write(struct.pack("<I", len(sections)))
    for name, arr in sections.items():
        arr = np.ascontiguousarray(arr)
        nb = name.encode()
        out.write(struct.pack("<I", len(nb)))
        out.write(nb)
        out.write(struct.pack("<IQ", _DT[arr.dtype], arr.nbytes))
        out.write(arr.tobytes())
        pad = (-out.tell()) % 8
        out.write(b"\0" * pad)
    return out.getvalue()


def blob_sections(blob: bytes) -> "OrderedDict[str, np.ndarray]":
    inv = {v: k for k, v in _DT.items()}
    assert blob[:8] == BLOB_MAGIC
    (n,) = struct.unpack_from("<I", blob, 8)
    off = 12
    out = OrderedDict()
    for _ in range(n):
        (ln,) = struct.unpack_from("<I", blob, off)
        off += 4
        name = blob[off:off + ln].decode()
        off += ln
        dt, nbytes = struct.unpack_from("<IQ", blob, off)
        off += 12
        out[name] = np.frombuffer(blob, dtype=inv[dt], count=nbytes // inv[dt].itemsize, offset=off).copy()
        off += nbytes
        off += (-off) % 8
    return out


@dataclass
class Compiled:
    rules: Rules
    scan_d: MealyDFA          # reverse relaxed detector prefilter
    scan_k: MealyDFA          # reverse exact context-keyword groups
    first: List[DFA]
    hot: List[DFA]
    hot_rules: List[HotRule]
    sections: "OrderedDict[str, np.ndarray]"
    blob: bytes
    scan_groups: List[List[int]] = None     # pattern ids of each SCAN group (group 0 first)


SCAN_BUDGET = 3     # prefix characters per detector pattern in the SCAN prefilter


def _acc_tables(m: MealyDFA):
    """acc_off/acc_ids flattening of a Mealy DFA's accept sets (index 0 = empty)."""
    off = np.zeros(len(m.acc_sets) + 1, dtype=np.uint32)
    ids: List[int] = []
    for i, s in enumerate(m.acc_sets):
        ids.extend(s)
        off[i + 1] = len(ids)
    return off, np.array(ids or [0], dtype=np.uint16)


SCAN_LDS_BYTES = 65536          # k_scan tables: u16 LDS byte addresses (class map + D rows + K rows)
SCAN_CMAP_BYTES = 1024
SCAN_GROUP_BYTES = 62 * 1024    # D table of a scan group >= 1 that keeps 16-bit byte addresses (two
                                # k_scan workgroups per CU); its K is a 1-row never-accepting stub
SCAN_WIDE_BYTES = 124 * 1024    # a WIDE group >= 1 (engine: rows padded to 4 entries, entries = offset / 2,
                                # one workgroup per CU): up to 64k transitions
SPILL_PREFIX = 10               # prefix of the built-ins moved out of group 0 (plan_scan_groups)
SCAN_GROUPS_MAX = 8             # k_pairs_merge merges at most this many per-group event lists per lane
DICT_SCAN_PREFIX = 4            # SCAN prefix of dictionary infoTypes (Rules)


def _table_bytes(m: MealyDFA) -> int:
    return m.n_states * ((m.n_classes + 2) & ~1) * 2


def _table_bytes_wide(m: MealyDFA) -> int:
    return m.n_states * ((m.n_classes + 4) & ~3) * 2


def _scan_dfa(patterns: Sequence[Pattern], budget: int, max_bytes: Optional[int] = None,
              prefixes: bool = True) -> Optional[MealyDFA]:
    """prefixes: honour the detectors' scan_prefix (longer relaxed prefixes: fewer candidate pairs,
    more states); without, every pattern keeps `budget` characters."""
    nd = NFA()
    sd = [add_relaxed(nd, p.pattern, p.pid, (p.scan_prefix if prefixes else None) or budget, reverse=True)
          for p in patterns]
    try:
        m = build_mealy_dfa(nd, sd, max_bytes=max_bytes)
    except RuleError:
        if max_bytes is None:
            raise
        return None
    return m if max_bytes is None or _table_bytes(m) <= max_bytes else None


def _scan_dfa_fit(patterns: Sequence[Pattern], budget: int, max_bytes: int) -> Optional[MealyDFA]:
    """the automaton with the declared scan prefixes, else (too large) with `budget` for every pattern"""
    m = _scan_dfa(patterns, budget, max_bytes)
    if m is None and any(p.scan_prefix for p in patterns):
        m = _scan_dfa(patterns, budget, max_bytes, prefixes=False)
    return m


def _prefix_key(p: Pattern) -> str:
    return re.sub(r"^\(\?i\)|\\b", "", p.pattern).lower()


def plan_scan_groups(rules: Rules, budget: int, k_bytes: int) -> List[Tuple[List[Pattern], MealyDFA]]:
    """Split the detector patterns over reverse D automata that each fit k_scan's LDS (config 5: 500+
    custom types).  One automaton per independent pattern set multiplies the states (a product of
    the sets' tries), so large rule sets get several smaller automata, each stepped by its own
    k_scan pass.  Group 0 is stepped together with the keyword automaton K and holds every built-in
    and excluder pattern; the rest, ordered by prefix so that similar prefixes share states, is cut
    in halves until each half fits."""
    limit0 = SCAN_LDS_BYTES - SCAN_CMAP_BYTES - k_bytes
    whole = _scan_dfa_fit(rules.patterns, budget, limit0) if len(rules.patterns) <= 256 else None
    if whole is not None:
        return [(list(rules.patterns), whole)]
    excl = set()
    for insp in rules.variants():
        for rs in insp.get("rule_set", []) or []:
            for rule in rs.get("rules", []):
                if "exclusion_rule" in rule:
                    excl |= {it["name"] for it in rule["exclusion_rule"].get("exclude_info_types", {}).get(
                        "info_types", [])}
    base = [p for p in rules.patterns if not p.custom or p.type_name in excl]
    rest = sorted((p for p in rules.patterns if p.custom and p.type_name not in excl), key=_prefix_key)
    # group 0 keeps the declared prefixes: when they do not fit beside K (config 5's larger keyword
    # automaton), the non-excluder built-ins with the longest declared prefixes move to a group of their
    # own (one more k_scan pass) rather than every built-in falling back to `budget` characters --
    # short digit-run prefixes fire at every digit run of the custom types' ids
    spill: List[Pattern] = []
    g0 = _scan_dfa(base, budget, limit0)
    if g0 is None:
        spill = [p for p in base if p.type_name not in excl and p.scan_prefix]
        base = [p for p in base if not (p.type_name not in excl and p.scan_prefix)]
        g0 = _scan_dfa(base, budget, limit0) if base else None
    if g0 is None:
        spill, base = [], spill + base
        base.sort(key=lambda p: p.pid)
        g0 = _scan_dfa_fit(base, budget, limit0)
    if g0 is None:
        raise RuleError("the built-in detectors' SCAN automaton does not fit k_scan's LDS")
    out = [(base, g0)]

    def fits(m, wide):
        return m is not None and (_table_bytes(m) <= SCAN_GROUP_BYTES or
                                  (wide and _table_bytes_wide(m) <= SCAN_WIDE_BYTES and
                                   m.n_states * ((m.n_classes + 4) & ~3) <= 65536))

    def split(pats):
        # the declared prefixes (dictionary types: DICT_SCAN_PREFIX) are worth a split -- they cut the
        # candidate pairs several-fold -- so a set is halved before its prefixes are shortened.  A set
        # whose automaton fits a WIDE table stays one group (one k_scan workgroup per CU: 352 us per
        # pass at config 5 against 283 for a narrow pass, so one wide pass beats two narrow ones); only
        # a set too large for that is halved.  A single pattern whose automaton does not fit falls back
        # to `budget` characters.
        m = _scan_dfa(pats, budget, SCAN_WIDE_BYTES)
        if fits(m, True):
            out.append((pats, m))
            return
        if len(pats) == 1:
            m = _scan_dfa(pats, budget, SCAN_WIDE_BYTES, prefixes=False)
            if not fits(m, True):
                raise RuleError(f"the SCAN automaton of {pats[0].type_name} alone does not fit k_scan's LDS")
            out.append((pats, m))
            return
        h = len(pats) // 2
        split(pats[:h])
        split(pats[h:])
    if spill:
        # the spilled built-ins have a table of their own: their prefixes may grow to SPILL_PREFIX
        # (digit-run detectors: a 7-digit prefix still fires at every 7-9 digit custom id)
        long = [dataclasses.replace(p, scan_prefix=max(p.scan_prefix, SPILL_PREFIX)) for p in spill]
        m = _scan_dfa(long, budget, SCAN_GROUP_BYTES)
        if m is not None:
            out.append((sorted(long, key=lambda p: p.pid), m))
        else:
            split(sorted(spill, key=lambda p: p.pid))
    if rest:
        split(rest)
    if len(out) > SCAN_GROUPS_MAX:
        raise RuleError(f"{len(out)} SCAN groups (more than {SCAN_GROUPS_MAX})")
    return out


def compile_rules(rules: Rules, scan_budget: int = SCAN_BUDGET) -> Compiled:
    P = len(rules.patterns)
    G = len(rules.kw_groups)
    if P == 0:
        raise RuleError("no detectors")
    # ---- SCAN (two Mealy automata stepped together, right to left) ----
    nk = NFA()
    sk = [add_relaxed(nk, pat, g, 0, reverse=True) for g, (_t, pat, _a) in enumerate(rules.kw_groups) if pat]
    if not sk:                       # no keywords: a one-state automaton that never accepts
        sk = [add_relaxed(nk, "\\xff\\x00\\xff", 0, 0, reverse=True)]
    scan_k = build_mealy_dfa(nk, sk)
    groups = plan_scan_groups(rules, scan_budget, _table_bytes(scan_k))
    scan_d = groups[0][1]
    for _, m in groups:
        if m.n_classes + 1 > 255:
            raise RuleError("too many byte classes")
    if scan_k.n_classes + 1 > 255:
        raise RuleError("too many byte classes")
    cmap2 = scan_d.cmap.astype(np.uint16) | (scan_k.cmap.astype(np.uint16) << 8)
    k_off, k_ids = _acc_tables(scan_k)

    # ---- FIRST: one anchored leftmost-first DFA per detector pattern ----
    first = []
    min_len = 1 << 30
    # window_ok: no detector can consume '\n' or test a text edge (\A, \Z).  Then no match crosses
    # the "\n" that joins a re-scan window, and a match inside one utterance is the same
    # match inside the window, which is what lets the engine re-scan windows incrementally.
    window_ok = 1
    for p in rules.patterns:
        n2 = NFA()
        st = add_pattern(n2, p.pattern, p.pid, reverse=False)
        first.append(build_first_dfa(n2, st))
        min_len = min(min_len, _min_len(parse(p.pattern)))
        for k, b, cs in zip(n2.kind, n2.b, n2.cs):
            if (k == CHAR and cs & NEWLINE) or (k == ASSERT and b in (A_BEGIN, A_END)):
                window_ok = 0

    # ---- variants (context merge, main.py:609-686) + HOT rule DFAs ----
    T = len(rules.type_names)
    V = 1 + G
    hot_rules: List[HotRule] = []
    hot_index: Dict[tuple, int] = {}
    var_enabled = np.zeros((V, T), dtype=np.uint8)
    var_minlik = np.zeros(V, dtype=np.uint8)
    rule_off = np.zeros(V * T + 1, dtype=np.uint32)
    rule_ids: List[int] = []
    excl_off = np.zeros(V * T + 1, dtype=np.uint32)
    excl_ids: List[int] = []
    for v, insp in enumerate(rules.variants()):
        enabled = {it.get("name") for it in insp.get("info_types", [])}
        enabled |= {c.get("info_type", {}).get("name") for c in insp.get("custom_info_types", []) or []}
        for name in list(enabled) + rules.external_types:
            if name in rules.type_id:
                var_enabled[v, rules.type_id[name]] = 1
        var_minlik[v] = lik_value(insp.get("min_likelihood", DEFAULT_MIN_LIKELIHOOD))
        per_type_rules = [[] for _ in range(T)]
        per_type_excl = [[] for _ in range(T)]
        for rs in insp.get("rule_set", []) or []:
            tnames = [it.get("name") for it in rs.get("info_types", [])]
            for rule in rs.get("rules", []):
                if "hotword_rule" in rule:
                    h = rule["hotword_rule"]
                    adj = h.get("likelihood_adjustment", {})
                    prox = h.get("proximity", {})
                    fixed = adj.get("fixed_likelihood")
                    hr = HotRule(h["hotword_regex"]["pattern"], int(prox.get("window_before", 0)),
                                 int(prox.get("window_after", 0)), 0 if fixed is None else lik_value(fixed),
                                 int(adj.get("relative_likelihood", 0)))
                    key = (hr.pattern, hr.window_before, hr.window_after, hr.fixed, hr.relative)
                    if key not in hot_index:
                        hot_index[key] = len(hot_rules)
                        hot_rules.append(hr)
                    for tn in tnames:
                        if tn in rules.type_id:
                            per_type_rules[rules.type_id[tn]].append(hot_index[key])
                elif "exclusion_rule" in rule:
                    ex = rule["exclusion_rule"]
                    mt = ex.get("matching_type", "MATCHING_TYPE_FULL_MATCH")
                    if mt != "MATCHING_TYPE_FULL_MATCH" or "exclude_info_types" not in ex:
                        raise RuleError("only exclude_info_types with MATCHING_TYPE_FULL_MATCH is supported")
                    xs = [it["name"] for it in ex["exclude_info_types"].get("info_types", [])]
                    for tn in tnames:
                        if tn in rules.type_id:
                            per_type_excl[rules.type_id[tn]].extend(rules.type_id[x] for x in xs if x in rules.type_id)
        for x in rules.external_types:
            xt = rules.type_id[x]
            if per_type_rules[xt] or per_type_excl[xt] or any(xt in l for l in per_type_excl):
                raise RuleError(f"external type {x} cannot be named by a hotword or exclusion rule")
        for t in range(T):
            rule_ids.extend(per_type_rules[t])
            rule_off[v * T + t + 1] = len(rule_ids)
            excl_ids.extend(per_type_excl[t])
            excl_off[v * T + t + 1] = len(excl_ids)
    # excluder patterns (their type is excluded-against in some variant) get a slot in the resolve
    # kernel's private state and come FIRST in every SCAN-D accept set, so that a same-start
    # excluder is known before the findings it may exclude (A.5).
    excluder_types = set(excl_ids[:int(excl_off[-1])])
    excluded_types = {t for v in range(V) for t in range(T) if excl_off[v * T + t + 1] > excl_off[v * T + t]}
    if excluder_types & excluded_types:
        raise RuleError("an infoType that is both excluded and excluding is not supported")
    exidx = np.full(P, 0xFF, dtype=np.uint8)
    ne = 0
    for p in rules.patterns:
        if rules.type_id[p.type_name] in excluder_types:
            exidx[p.pid] = ne
            ne += 1
    if ne > 8:
        raise RuleError("more than 8 excluder patterns")
    # one accept-set id space over all scan groups: group g's set a > 0 -> acc_base[g] + a
    acc_sets: List[Tuple[int, ...]] = [()]
    acc_base = []
    for _, m in groups:
        m.acc_sets = [tuple(sorted(s, key=lambda pid: (exidx[pid] == 0xFF, pid))) for s in m.acc_sets]
        acc_base.append(len(acc_sets) - 1)
        acc_sets.extend(m.acc_sets[1:])
    d_off = np.zeros(len(acc_sets) + 1, dtype=np.uint32)
    d_list: List[int] = []
    for i, st in enumerate(acc_sets):
        d_list.extend(st)
        d_off[i + 1] = len(d_list)
    d_ids = np.array(d_list or [0], dtype=np.uint16)

    def global_accid(g, m):
        a = m.acc_id.reshape(-1).astype(np.int64)
        return np.where(a > 0, a + acc_base[g], 0).astype(np.uint16)
    hot = []
    for hr in hot_rules:
        n3 = NFA()
        st = add_pattern(n3, hr.pattern, 0, reverse=False)
        hot.append(build_set_dfa(n3, [st], unanchored=True))
    hot_desc = np.zeros((max(1, len(hot_rules)), 4), dtype=np.int32)
    for i, hr in enumerate(hot_rules):
        hot_desc[i] = (hr.window_before, hr.window_after, hr.fixed, hr.relative)

    # ---- pools: FIRST + HOT tables in one global-memory pool ----
    pool_trans, pool_flags, pool_cmap = [], [], []
    tr_off = fl_off = cm_off = 0

    def put(d: DFA):
        nonlocal tr_off, fl_off, cm_off
        desc = (tr_off, fl_off, cm_off, d.n_classes + 1, d.start[0], d.start[1], d.start[2], d.n_states)
        pool_trans.append(d.trans.reshape(-1))
        pool_flags.append(d.flags)
        pool_cmap.append(d.cmap)
        tr_off += d.trans.size
        fl_off += d.flags.size
        cm_off += 256
        return desc

    first_desc = np.array([put(d) for d in first], dtype=np.int32).reshape(-1, 8)
    hot_dfa_desc = (np.array([put(d) for d in hot], dtype=np.int32).reshape(-1, 8) if hot
                    else np.zeros((1, 8), np.int32))
    if tr_off >= (1 << 31):
        raise RuleError("table pool too large")

    names_blob = b"".join(n.encode("ascii") + b"\0" for n in rules.type_names)
    kw_type = np.array([rules.type_id[t] for t, _, _ in rules.kw_groups] or [0], dtype=np.uint16)
    kw_always = np.array([1 if a else 0 for _, _, a in rules.kw_groups] or [0], dtype=np.uint8)
    meta = np.array([P, G, T, V,
                     scan_d.n_states, scan_d.n_classes + 1, scan_d.start,
                     scan_k.n_states, scan_k.n_classes + 1, scan_k.start,
                     len(hot_rules), min_len, scan_budget, window_ok, len(groups) - 1, 0], dtype=np.int64)
    S = OrderedDict()
    S["meta"] = meta
    S["scan.cmap2"] = cmap2
    S["scan.d.trans"] = scan_d.trans.reshape(-1)
    S["scan.d.accid"] = global_accid(0, scan_d)
    S["scan.d.acc_off"] = d_off
    S["scan.d.acc_ids"] = d_ids
    S["scan.k.trans"] = scan_k.trans.reshape(-1)
    S["scan.k.accid"] = scan_k.acc_id.reshape(-1).astype(np.uint16)
    S["scan.k.acc_off"] = k_off
    S["scan.k.acc_ids"] = k_ids
    S["det.type"] = np.array([rules.type_id[p.type_name] for p in rules.patterns], dtype=np.uint16)
    S["det.validator"] = np.array([VALIDATOR_IDS[p.validator] for p in rules.patterns], dtype=np.uint8)
    S["det.lik"] = np.array([p.likelihood for p in rules.patterns], dtype=np.uint8)
    S["det.exidx"] = exidx
    S["det.first_desc"] = first_desc.reshape(-1)
    S["hot.rule"] = hot_desc.reshape(-1)
    S["hot.dfa_desc"] = hot_dfa_desc.reshape(-1)
    S["pool.trans"] = np.concatenate(pool_trans).astype(np.uint16) if pool_trans else np.zeros(1, np.uint16)
    S["pool.flags"] = np.concatenate(pool_flags).astype(np.uint8) if pool_flags else np.zeros(1, np.uint8)
    S["pool.cmap"] = np.concatenate(pool_cmap).astype(np.uint8) if pool_cmap else np.zeros(256, np.uint8)
    S["var.enabled"] = var_enabled.reshape(-1)
    S["var.minlik"] = var_minlik
    S["var.rule_off"] = rule_off
    S["var.rule_ids"] = np.array(rule_ids or [0], dtype=np.uint16)
    S["var.excl_off"] = excl_off
    S["var.excl_ids"] = np.array(excl_ids or [0], dtype=np.uint16)
    S["kw.type"] = kw_type
    S["kw.always"] = kw_always
    S["types.names"] = np.frombuffer(names_blob, dtype=np.uint8).copy()
    # scan groups >= 1 (config-5 scale): (states, classes + EOT, start) + class map, table, accept ids
    if len(groups) > 1:
        S["scan.groups"] = np.array([[m.n_states, m.n_classes + 1, m.start, 0] for _, m in groups[1:]],
                                    dtype=np.int64).reshape(-1)
        for g, (_, m) in enumerate(groups[1:], start=1):
            S[f"scan.g{g}.cmap"] = m.cmap.astype(np.uint8)
            S[f"scan.g{g}.trans"] = m.trans.reshape(-1)
            S[f"scan.g{g}.accid"] = global_accid(g, m)
    blob = _sections_to_blob(S)
    return Compiled(rules, scan_d, scan_k, first, hot, hot_rules, S, blob, [[p.pid for p in ps] for ps, _ in groups])


def _min_len(tree) -> int:
    def ml(items):
        return sum(one(op, av) for op, av in items)

    def one(op, av):
        if op in (C.LITERAL, C.NOT_LITERAL, C.ANY, C.IN):
            return 1
        if op == C.AT:
            return 0
        if op == C.SUBPATTERN:
            return ml(av[-1])
        if op == C.BRANCH:
            return min(ml(b) for b in av[1])
        if op in (C.MAX_REPEAT, C.MIN_REPEAT):
            return av[0] * ml(av[2])
        return 0
    return max(1, ml(list(tree)))


_CACHE: Dict[str, Compiled] = {}


def compile_default(dlp_config_path: Optional[str] = None, builtin_path: Optional[str] = None,
                    cache_dir: Optional[str] = None) -> Compiled:
    rules = Rules.load(dlp_config_path, builtin_path)
    key = hashlib.sha256(json.dumps([rules.raw, [p.__dict__ for p in rules.patterns]], sort_keys=True,
                                    default=str).encode()).hexdigest()[:16]
    if key in _CACHE:
        return _CACHE[key]
    c = compile_rules(rules)
    _CACHE[key] = c
    return c


if __name__ == "__main__":
    import time
    t0 = time.time()
    c = compile_default()
    m = c.sections["meta"]
    print(f"compiled in {time.time() - t0:.1f}s; SCAN-D {c.scan_d.n_states}x{c.scan_d.n_classes + 1} "
          f"SCAN-K {c.scan_k.n_states}x{c.scan_k.n_classes + 1} "
          f"({(c.sections['scan.d.trans'].nbytes + c.sections['scan.k.trans'].nbytes) / 1024:.1f} KiB LDS); "
          f"FIRST states {[d.n_states for d in c.first]}; HOT {[d.n_states for d in c.hot]}; "
          f"pool {c.sections['pool.trans'].nbytes / 1024:.1f} KiB; blob {len(c.blob) / 1024:.1f} KiB")
