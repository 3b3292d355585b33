"""The reference's own callers of the trainer bind to heist_amd's signatures unchanged.

The call sites are recorded here as data (argument names as the reference passes them):
main.py:32-49 (cmd_train) and visualization/server.py:50-68, :145-146, :163, :220-230,
:278, :298, :318, :328.  inspect.signature().bind checks that every call is accepted by
heist_amd's AdversarialTrainer / EnvironmentConfig as written; the attributes the server
reads and writes are checked on the class's __init__ source (no GPU needed)."""
import inspect

from heist_amd.environment import EnvironmentConfig
from heist_amd.training import AdversarialTrainer

# (callable name, positional args, keyword args) as the reference writes them
CALLS = [
    ("EnvironmentConfig", (), dict(grid_rows=20, grid_cols=20, max_steps=200, start_pos=(1, 1), vault_pos=(18, 18),
                                   architect_budget=8)),  # main.py:32-39
    ("EnvironmentConfig", (), dict(grid_rows=20, grid_cols=20, start_pos=(1, 1), vault_pos=(18, 18))),  # server.py:50
    ("AdversarialTrainer", (), dict(config=None, total_episodes=500, solver_episodes_per_layout=20, save_dir="c",
                                    log_dir="l")),  # main.py:41-47, server.py:57-63
    ("train", (), dict(resume=True)),  # main.py:49
    ("train", (), dict(callback=print, resume=False)),  # server.py:163
    ("find_latest_checkpoint", (), {}),  # server.py:66
    ("resume_from_checkpoint", (), {}),  # server.py:68
    ("get_game_log", (), {}),  # server.py:168
    ("run_interactive_episodes", (), dict(num_episodes=5, budget=15, freeze_architect=False, freeze_solver=False,
                                          temperature=1.0, solver_attempts=3, allow_cameras=True,
                                          allow_guards=True, callback=print)),  # server.py:220-230
    ("simulate_episode", (), dict(budget=15, solver_attempts=1)),  # server.py:278, :328
    ("list_checkpoints", (), {}),  # server.py:298
    ("load_checkpoint", (50,), {}),  # server.py:318
]

# attributes server.py reads or assigns on the trainer (:145-146, :158-159, :167, :235)
ATTRS = ["total_episodes", "solver_episodes", "game_log", "global_episode"]


def test_reference_call_sites_bind():
    for name, args, kw in CALLS:
        if name == "EnvironmentConfig":
            inspect.signature(EnvironmentConfig).bind(*args, **kw)
        elif name == "AdversarialTrainer":
            inspect.signature(AdversarialTrainer.__init__).bind(None, *args, **kw)
        else:
            inspect.signature(getattr(AdversarialTrainer, name)).bind(None, *args, **kw)


def test_reference_trainer_attributes():
    src = inspect.getsource(AdversarialTrainer.__init__) + inspect.getsource(AdversarialTrainer)
    for a in ATTRS:
        assert "self.%s =" % a in src or "self.%s=" % a in src, a
