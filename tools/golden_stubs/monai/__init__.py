transforms = None
