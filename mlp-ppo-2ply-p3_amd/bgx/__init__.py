"""bgx — MI355X-native backgammon self-play engine: a drop-in for the reference's
env / board / move / agent hot path."""
from .engine import Engine, encode  # noqa: F401
from .types import (Player, Position, SubMove, FullMove, BoardState, ImmutableBoard,  # noqa: F401
                    get_all_possible_moves, filter_full_moves_by_max_submoves, generate_all_board_features,
                    get_board_features_batch_from_tensors, execute_full_move_on_board_copy,
                    execute_sub_move_on_board, board_hash, board_to_string, get_all_dice_rolls_tensor)
from .env import BackgammonEnv, VectorizedBackgammonEnv  # noqa: F401
from .policy import PolicyNet  # noqa: F401

BackgammonPolicyNetwork = PolicyNet
