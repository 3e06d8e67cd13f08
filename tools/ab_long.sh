set -o pipefail
R=$PWD; O=$R/gpurun_out/ab_long; mkdir -p $O
for i in 1 2; do
  PII_LIB=$R/exp_libs/libpii_old.so timeout -k 10 200 python -u bench.py --workload long --no-cpu-baseline > $O/old$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --workload long --no-cpu-baseline > $O/new$i.json 2>/dev/null || exit 1
  PII_NER_LIB=$R/exp_libs/libner_base.so timeout -k 10 200 python -u bench.py --workload ner > $O/nerold$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --workload ner > $O/nernew$i.json 2>/dev/null || exit 1
done
echo AB_DONE
