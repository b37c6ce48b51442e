set -e
bash tools/kstats.sh c3final > gpurun_out/kfinal_c3.txt
CFG=c5 bash tools/kstats.sh c5final > gpurun_out/kfinal_c5.txt
cat gpurun_out/kfinal_c3.txt; echo; cat gpurun_out/kfinal_c5.txt
