# round 4: where the 10:3 decode loses against the streaming rate: the same kernel on every erasure pattern
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4f; mkdir -p $O
for e in data random none; do
  AB_ERASE=$e timeout -k 10 120 python tools/ab_one.py 10 13 1400 1048576 >> $O/erase_103.txt 2>&1 || { cat $O/erase_103.txt; exit 1; }
  AB_ERASE=$e timeout -k 10 120 python tools/ab_one.py 10 13 1408 1048576 >> $O/erase_103.txt 2>&1 || { cat $O/erase_103.txt; exit 1; }
done
AB_ERASE=data timeout -k 10 120 python tools/ab_one.py 20 23 1440 1048576 >> $O/erase_103.txt 2>&1
cat $O/erase_103.txt
