"""AlphaGo.training.reinforcement_value_trainer (empty in the reference) — value-net training.
See rocalphago_amd/training/value_trainer.py."""
from rocalphago_amd.training.value_trainer import (generate_value_dataset,  # noqa: F401
                                                   run_training)

if __name__ == '__main__':
    run_training()
