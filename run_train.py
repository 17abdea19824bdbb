"""Training entry point with the reference's CLI (run_train.py:20-121):

    python run_train.py -yaml_path experiment_conf/example.yaml [-max_iters N]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 run_train.py -yaml_path experiment_conf/c4_train.yaml

The graph filter's forward and reverse run on the HIP kernels (irdu_amd); one process per GPU,
gradients averaged with bucketed RCCL all-reduces.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    from irdu_amd import training
    training.main()
