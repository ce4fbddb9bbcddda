require "./app"
run Sinatra::Application
