from .optimizers import (SGD, Adadelta, Adam, KVariable, Nadam, Optimizer, RMSprop, deserialize, get,
                         get_value, serialize, set_value)

__all__ = ["SGD", "RMSprop", "Adadelta", "Adam", "Nadam", "Optimizer", "KVariable", "get",
           "get_value", "set_value", "serialize", "deserialize"]
