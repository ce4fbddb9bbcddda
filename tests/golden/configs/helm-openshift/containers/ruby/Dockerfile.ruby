FROM ruby:2.5
COPY . /app
WORKDIR /app
RUN bundle install
EXPOSE 8080
CMD ["ruby","/app/app.rb"]
