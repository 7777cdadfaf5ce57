# round-4 batch 23: decode layer kernels' residency A/B (LDS padding caps workgroups per CU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  timeout -k 10 240 python -u bench/decode_bench.py --batches 1 --decode-only 200 2>gpurun_out/dec_ab.err | tail -1 | cut -c1-100 || { tail -20 gpurun_out/dec_ab.err; return 1; }
  echo "  ($*)"
}
KCA_DECODE_MERGED=0 run base &&
KCA_DECODE_MERGED=0 KCA_DEC_LDS_PAD=40960,0 run k2 3/CU &&
KCA_DECODE_MERGED=0 KCA_DEC_LDS_PAD=57344,0 run k2 2/CU &&
KCA_DECODE_MERGED=0 KCA_DEC_LDS_PAD=0,40960 run k3 3/CU &&
KCA_DECODE_MERGED=0 KCA_DEC_LDS_PAD=0,57344 run k3 2/CU &&
KCA_DECODE_MERGED=1 KCA_DEC_LDS_PAD=40960,0 run merged 3/CU &&
KCA_DECODE_MERGED=1 KCA_DEC_LDS_PAD=57344,0 run merged 2/CU &&
KCA_DECODE_MERGED=0 run base
