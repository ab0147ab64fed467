set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 env "$@" > gpurun_out/tlb_$tag.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/tlb_$tag.log; exit 1; }; python3 -c "import json; d=json.loads(open('gpurun_out/tlb_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e6,1), 'M', round(d['ms_per_step'],4), 'ms load', round(d['table_load'],3))"; }
for r in 1 2; do
run lr_def XFLOW_CONTIG=0 python bench.py --steps 30 --warmup 5
run lr_contig XFLOW_CONTIG=1 python bench.py --steps 30 --warmup 5
run lr_cap28 XFLOW_CONTIG=0 python bench.py --steps 30 --warmup 5 --log2-cap 28 --table-load 0.47
run fm_def XFLOW_CONTIG=0 python bench.py --steps 30 --warmup 5 --model fm --v-dim 8
run fm_contig XFLOW_CONTIG=1 python bench.py --steps 30 --warmup 5 --model fm --v-dim 8
run fm_cap28 XFLOW_CONTIG=0 python bench.py --steps 30 --warmup 5 --model fm --v-dim 8 --log2-cap 28 --table-load 0.47
done
