set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05_segtl; mkdir -p $O
NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_tl.so timeout -k 10 200 python tools/seg_tl.py > $O/tl.jsonl 2> $O/tl.err || { tail -20 $O/tl.err; exit 1; }
cat $O/tl.jsonl
