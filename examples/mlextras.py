"""``from mlextras import IPyParallelLogger, configure_session`` (engine-side helpers)."""
import _path  # noqa: F401
from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger, configure_session  # noqa: F401
