# Host paths, library lane policy vs NOISE_AEAD_LANES=narrow, same box.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/hostab; mkdir -p $O
for pol in auto narrow; do
  if [ $pol = narrow ]; then export NOISE_AEAD_LANES=narrow; fi
  timeout -k 10 300 python tools/e2e.py > $O/e2e_c2_$pol.json 2> $O/err || { tail -20 $O/err; exit 1; }
  timeout -k 10 300 python tools/e2e.py --cipher aesgcm > $O/e2e_c3_$pol.json 2> $O/err || { tail -20 $O/err; exit 1; }
  timeout -k 10 300 python tools/wire_e2e.py > $O/wire_c2_$pol.jsonl 2> $O/err || { tail -20 $O/err; exit 1; }
  timeout -k 10 300 python tools/wire_e2e.py --cipher aesgcm > $O/wire_c3_$pol.jsonl 2> $O/err || { tail -20 $O/err; exit 1; }
  timeout -k 10 300 python tools/echo_loopback.py > $O/echo_$pol.json 2> $O/err || { tail -20 $O/err; exit 1; }
done
