"""Small runtime utilities: finite-output checking, device timing, environment report."""
from .runtime import check_finite, env_report, finite_checks, strict_mode, time_fn  # noqa: F401
