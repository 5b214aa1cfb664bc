mkdir -p gpurun_out/r05v
for v in 1200 1500; do for g in 0 1; do
  MCC_GROUP=$g timeout -k 10 120 python3 bench.py --config config4 --views $v --no-cpu --no-parity --no-extra --steps 1000 --warmup 50 > gpurun_out/r05v/b.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r05v/b.json')); print('config4 views', sys.argv[1], 'MCC_GROUP', sys.argv[2], round(d['ms_per_step']*1e3,2))" $v $g
done; done
for g in 0 1; do
  MCC_GROUP=$g timeout -k 10 120 python3 bench.py --config config5 --views 1000 --no-cpu --no-parity --no-extra --steps 1000 --warmup 50 > gpurun_out/r05v/b.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r05v/b.json')); print('config5 views 1000 MCC_GROUP', sys.argv[1], round(d['ms_per_step']*1e3,2))" $g
done
