"""Model registry — drop-in for the reference's models/__init__.py (lines 4-44):
`--model <name>` resolves to module `models.<name>_model` and the BaseModel subclass whose
lower-cased name equals `<name without underscores>model`.  An unknown name prints the same
hint and exits with status 0, as the reference does."""
import importlib

from models.base_model import BaseModel


def find_model_using_name(model_name):
    module_name = "models." + model_name + "_model"
    lib = importlib.import_module(module_name)
    wanted = model_name.replace('_', '') + 'model'
    found = None
    for attr, obj in vars(lib).items():
        if attr.lower() == wanted.lower() and isinstance(obj, type) and issubclass(obj, BaseModel):
            found = obj
    if found is None:
        print("In %s.py, there should be a subclass of BaseModel with class name that matches %s in lowercase."
              % (module_name, wanted))
        exit(0)
    return found


def get_option_setter(model_name):
    return find_model_using_name(model_name).modify_commandline_options


def create_model(opt):
    cls = find_model_using_name(opt.model)
    instance = cls()
    instance.initialize(opt)
    print("model [%s] was created" % (instance.name()))
    return instance
