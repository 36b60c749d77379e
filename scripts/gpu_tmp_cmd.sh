TAG=r03lipu KNOB=ERP_LIP2 VALUES="1" TEST_K="consensus or find or manual or shard" bash scripts/gpu_ab_prof.sh
