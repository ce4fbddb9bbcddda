module example.com/hello

go 1.15
