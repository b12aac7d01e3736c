"""AlphaGo.preprocessing.game_converter — SGF -> HDF5. See rocalphago_amd/features/converter.py."""
from rocalphago_amd.features.converter import (GameConverter, SizeMismatchError,  # noqa: F401
                                               run_game_converter)

if __name__ == '__main__':
    run_game_converter()
