#!/bin/bash
# end_to_end (1024^2 x 500 march + D2H + .npy) with 1 and 8 writer threads
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for w in 1 8 1 8; do
  BURG_NPY_WRITERS=$w timeout -k 10 120 python -c "import bench, json; print('writers $w', json.dumps(bench.end_to_end()))" 2>/dev/null | grep writers | cut -c1-120
done
