from . import collectives  # noqa: F401
from .comm import Communicator, Workers  # noqa: F401
from .events import Event, EventQueue, EventType  # noqa: F401
