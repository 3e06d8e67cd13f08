"""A/B timing of ner_gemm builds (BERT-base shapes, 64 x 128 tokens) beside torch.nn.functional.linear
(hipBLASLt), with a numerics check of every build against torch.  Each build is its own CDLL
(ner.open_library), timed in ROUNDS interleaved rounds (the minimum is reported, so clock ramp-up and
order do not favour one build).  usage: python tools/gemm_ab.py LIB..."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "context-based-pii_amd"))
import ner  # noqa: E402

TOKENS = int(os.environ.get("GEMM_M", "8192"))     # 64 x 128 tokens (bench --workload ner); 524288 = ner-redact
SHAPES = [("qkv", TOKENS, 2304, 768, 0), ("out", TOKENS, 768, 768, 2), ("ffn1", TOKENS, 3072, 768, 1),
          ("ffn2", TOKENS, 768, 3072, 2)]


ROUNDS = 5


def timeit(fn, reps=max(3, 50 * 8192 // TOKENS)):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3     # us


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {}
    for name, M, N, K, epi in SHAPES:
        A = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
        W = (torch.randn(N, K, generator=g) * 0.05).to(dev, torch.bfloat16)
        b = torch.randn(N, generator=g).to(dev)
        R = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ref = torch.nn.functional.linear(A.float(), W.float(), b)
        if epi == 1:
            ref = torch.nn.functional.gelu(ref)
        elif epi == 2:
            ref = ref + R.float()
        flop = 2.0 * M * N * K
        libs = [(os.path.basename(p), ner.open_library(os.path.join(ROOT, p))) for p in sys.argv[1:]]
        st = torch.cuda.current_stream().cuda_stream
        best = {n: float("inf") for n, _ in libs}
        best["torch"] = float("inf")
        errs = {}
        for _ in range(ROUNDS):
            best["torch"] = min(best["torch"], timeit(lambda: torch.nn.functional.linear(A, W, b.to(torch.bfloat16))))
            for n, lib in libs:
                def run(lib=lib):
                    rc = lib.ner_gemm(A.data_ptr(), W.data_ptr(), b.data_ptr(), R.data_ptr(), C.data_ptr(), M, N, K,
                                      epi, st)
                    assert rc == 0
                if n not in errs:
                    run()
                    torch.cuda.synchronize()
                    errs[n] = ((C.float() - ref).norm() / ref.norm()).item()
                best[n] = min(best[n], timeit(run))
        row = {"torch_linear_us": round(best["torch"], 1)}
        for n, _ in libs:
            row[n] = {"us": round(best[n], 1), "tflops": round(flop / best[n] / 1e6, 1), "rel_l2": round(errs[n], 5)}
        row["torch_tflops"] = round(flop / row["torch_linear_us"] / 1e6, 1)
        res[name] = row
        print(name, json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
