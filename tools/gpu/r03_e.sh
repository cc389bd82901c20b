# round 3: hard-limit GPU tests (replay fix) then the profiling set (tools/gpu/r03_c.sh)
cd /root/repo
bash tools/gpu/r03_d.sh
bash tools/gpu/r03_c.sh
exit 0
