# End-to-end host paths only (batch API, wire path, TCP echo): gpurun_out/host/.
set -eu
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/host; mkdir -p $O
timeout -k 10 300 python tools/e2e.py > $O/e2e_c2.json 2> $O/e2e_c2.err || { tail -20 $O/e2e_c2.err; exit 1; }
timeout -k 10 300 python tools/e2e.py --cipher aesgcm > $O/e2e_c3.json 2> $O/e2e_c3.err || { tail -20 $O/e2e_c3.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py > $O/wire_c2.jsonl 2> $O/wire_c2.err || { tail -20 $O/wire_c2.err; exit 1; }
timeout -k 10 300 python tools/wire_e2e.py --cipher aesgcm > $O/wire_c3.jsonl 2> $O/wire_c3.err || { tail -20 $O/wire_c3.err; exit 1; }
timeout -k 10 300 python tools/echo_loopback.py > $O/echo.json 2> $O/echo.err || { tail -20 $O/echo.err; exit 1; }
cat $O/e2e_c2.json $O/e2e_c3.json $O/wire_c2.jsonl $O/wire_c3.jsonl $O/echo.json
