# Diagnostic: collect non-converged environments over many large synthetic batches.
mkdir -p gpurun_out
for cfg in "unitree_go2 65536 2 standing ones" "unitree_go2 65536 3 standing ones" \
           "unitree_go2 65536 4 tumbling ones" "unitree_go2 65536 5 tumbling bernoulli" \
           "unitree_go2 65536 6 standing bernoulli" "walter_sr 32768 2 standing ones" \
           "walter_sr 32768 3 tumbling bernoulli" "walter_sr_wheels 32768 4 tumbling bernoulli"; do
  timeout -k 5 120 python tools/find_stalls.py $cfg || exit 1
done
