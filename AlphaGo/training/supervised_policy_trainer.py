"""AlphaGo.training.supervised_policy_trainer — see rocalphago_amd/training/supervised.py."""
from rocalphago_amd.training.supervised import (BOARD_TRANSFORMATIONS,  # noqa: F401
                                                MetadataWriterCallback, one_hot_action,
                                                run_training, shuffled_hdf5_batch_generator)

if __name__ == '__main__':
    run_training()
