"""AlphaGo.training.reinforcement_policy_trainer — see rocalphago_amd/training/reinforcement.py."""
from rocalphago_amd.training.reinforcement import (_make_training_pair, log_loss,  # noqa: F401
                                                   run_n_games, run_training)

if __name__ == '__main__':
    run_training()
