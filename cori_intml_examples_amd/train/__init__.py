from . import callbacks
from .callbacks import (Callback, CallbackList, CSVLogger, EarlyStopping, History, LambdaCallback,
                        LearningRateScheduler, ModelCheckpoint, ProgbarLogger, ReduceLROnPlateau,
                        TerminateOnNaN)
